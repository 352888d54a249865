#!/bin/bash
# Build-and-test matrix for beforeholiday_amd: for each PyTorch-ROCm base image, build the image
# (docker/Dockerfile: gfx950 extension build + CPU test suite) and report a pass / fail table.
#   scripts/ci_build.sh [image ...]         (default: the images below)
#   CI_LOCAL=1 scripts/ci_build.sh          (no docker: build + CPU tests in this environment)
#   CI_GPU=1 ...                            (also run the GPU tests in each image, needs /dev/kfd)
set -u
cd "$(dirname "$0")/.."
if [ "${CI_LOCAL:-0}" = "1" ]; then
  python -c "import __graft_entry__ as g; g.build()" && python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider
  rc=$?
  if [ $rc -eq 0 ] && [ "${CI_GPU:-0}" = "1" ]; then
    python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
    rc=$?
  fi
  exit $rc
fi
images=("$@")
[ ${#images[@]} -eq 0 ] && images=("rocm/pytorch:latest" "rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.8.0")
declare -A status
fail=0
for img in "${images[@]}"; do
  tag="bh-amd-ci:$(echo "$img" | tr '/:' '__')"
  echo "=== $img"
  if docker build -f docker/Dockerfile --build-arg FROM_IMAGE="$img" -t "$tag" .; then
    status[$img]=build-ok
    if [ "${CI_GPU:-0}" = "1" ]; then
      if docker run --rm --device=/dev/kfd --device=/dev/dri --group-add video --ipc=host \
           -e HSA_ENABLE_IPC_MODE_LEGACY=0 "$tag" \
           python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider; then
        status[$img]=gpu-ok
      else
        status[$img]=gpu-FAIL; fail=1
      fi
    fi
  else
    status[$img]=build-FAIL; fail=1
  fi
done
echo "=== summary"
for img in "${images[@]}"; do printf '%-80s %s\n' "$img" "${status[$img]}"; done
exit $fail

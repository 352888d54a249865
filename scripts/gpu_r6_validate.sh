#!/bin/bash
# round-6 validation on one MI355X: gpu-marked suite, smoke(), 1-GPU bench (scripts/gpu_full.sh), then the
# build-free smoke entry point the driver runs
export TMPDIR=/tmp
bash scripts/gpu_full.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
src=$?
tail -2 gpurun_out/smoke.log
exit $(( rc > src ? rc : src ))

#!/bin/bash
# rocprofv3 kernel summary of the ResNet-50 headline bench (3 steps after the stem marker)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/prof_resnet
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet -o run -- python bench.py --steps 8 --warmup 4 > gpurun_out/prof_resnet.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_resnet k_stem_fwd 3 gpurun_out/resnet_summary.md
rc=$?
rm -rf gpurun_out/prof_resnet
exit $rc

#!/bin/bash
# direct 3x3 plain / statistics epilogues branch-free (out-of-range stores, masked statistics) vs bounds-check branches
# new build vs ab/_C_base.so on the conv bench and the ResNet bench
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv3x3.py tests/test_conv_bn.py tests/test_resnet_fold.py > gpurun_out/t_c3bf.log 2>&1
rc=$?; tail -2 gpurun_out/t_c3bf.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_so.sh "python benchmarks/bench_conv3x3.py" c3bf || exit $?
bash scripts/ab_so.sh "python bench.py --steps 30 --warmup 8" c3bfrn || exit $?
for f in gpurun_out/c3bf_*.log; do echo "$f $(tail -1 $f)"; done
for f in gpurun_out/c3bfrn_*.log; do echo "$f $(tail -1 $f | cut -c1-100)"; done

#!/bin/bash
# direct 3x3 epilogue stores through a buffer resource (32-bit offsets) vs global stores: conv tests, then
# new build vs ab/_C_base.so on the conv bench and the ResNet bench
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv3x3.py tests/test_conv_bn.py tests/test_resnet_fold.py > gpurun_out/t_c3st.log 2>&1
rc=$?; tail -2 gpurun_out/t_c3st.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_so.sh "python benchmarks/bench_conv3x3.py" c3st || exit $?
bash scripts/ab_so.sh "python bench.py --steps 30 --warmup 8" c3rn || exit $?
for f in gpurun_out/c3st_*.log; do echo "$f $(tail -1 $f)"; done
for f in gpurun_out/c3rn_*.log; do echo "$f $(tail -1 $f | cut -c1-100)"; done

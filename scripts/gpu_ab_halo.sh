#!/bin/bash
# halo image-shift layout (new build) vs ab/_C_base.so: conv tests, then conv + ResNet bench A/B
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv3x3.py tests/test_conv_bn.py tests/test_dense.py tests/test_resnet_fold.py > gpurun_out/t_halo.log 2>&1
rc=$?; tail -2 gpurun_out/t_halo.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_so.sh "python benchmarks/bench_conv3x3.py" conv || exit $?
bash scripts/ab_so.sh "python bench.py --steps 30 --warmup 8" rn || exit $?
for f in gpurun_out/conv_*[12].log; do echo "$f $(grep -iE 'total|sum' $f | tail -2 | tr '\n' ' ')"; done
for f in gpurun_out/rn_*.log; do echo "$f $(tail -1 $f | cut -c1-100)"; done

#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv3x3.py tests/test_conv_bn.py > gpurun_out/t_nb.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/t_nb.log | head -3; [ $rc -ne 0 ] && exit $rc
BH_CONV3X3_NB=2 BH_CONV3X3_SW=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv3x3.py > gpurun_out/t_nb2.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/t_nb2.log | head -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python benchmarks/bench_conv3x3.py --ab > gpurun_out/conv_ab.log 2>&1 || exit $?
cat gpurun_out/conv_ab.log | grep rep
for v in "3 1" "2 0" "3 1" "2 0"; do set -- $v
  BH_CONV3X3_NB=$1 BH_CONV3X3_SW=$2 timeout -k 10 300 python bench.py --steps 30 --warmup 8 > gpurun_out/bench_nb$1.log 2>&1 || exit $?
  echo "nb=$1 sw=$2 $(tail -1 gpurun_out/bench_nb$1.log | cut -c1-110)"
done

#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_graph_checked.py > gpurun_out/t_gc.log 2>&1
grep -E "passed|failed|mismatch|loss_graph" gpurun_out/t_gc.log | head -8
timeout -k 10 300 python bench.py --steps 20 --warmup 6 > gpurun_out/bench_gc.log 2>&1 || exit $?
grep "\[bench\] {" gpurun_out/bench_gc.log; tail -1 gpurun_out/bench_gc.log
timeout -k 10 200 python benchmarks/bench_conv3x3.py > gpurun_out/conv_v3.log 2>&1 || exit $?
tail -1 gpurun_out/conv_v3.log
timeout -k 10 200 python benchmarks/bench_conv_s2.py > gpurun_out/convs2_v3.log 2>&1 || exit $?
tail -2 gpurun_out/convs2_v3.log

#!/bin/bash
# round-6 conv kernels vs MIOpen on the final tree: direct 3x3 (fwd / dgrad), stride-2 3x3, weight gradients
export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/bench_conv3x3.py > gpurun_out/r6_conv3x3.log 2>&1 || exit $?
tail -1 gpurun_out/r6_conv3x3.log
timeout -k 10 300 python benchmarks/bench_conv_s2.py > gpurun_out/r6_conv_s2.log 2>&1 || exit $?
tail -2 gpurun_out/r6_conv_s2.log
timeout -k 10 400 python benchmarks/bench_conv_wgrad.py > gpurun_out/r6_conv_wgrad.log 2>&1 || exit $?
tail -2 gpurun_out/r6_conv_wgrad.log

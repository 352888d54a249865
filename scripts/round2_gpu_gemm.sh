#!/bin/bash
# ping-pong GEMM: numerics of every tile kernel, then plain / fused timings vs hipBLASLt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_mfma.py > gpurun_out/gemm_test.log 2>&1 || { tail -30 gpurun_out/gemm_test.log; exit 1; }
tail -3 gpurun_out/gemm_test.log
timeout -k 10 300 python -u benchmarks/bench_gemm.py > gpurun_out/gemm_bench.log 2>&1 || { tail -30 gpurun_out/gemm_bench.log; exit 1; }
cat gpurun_out/gemm_bench.log

#!/bin/bash
# Offline GEMM solution search (utils/gemm_tuning.py): times every hipBLASLt / rocBLAS solution of each
# library GEMM signature of the ResNet-50 bench step and writes gpurun_out/tunableop_gfx950.csv, then
# A/B-measures the bench with the new table against hipBLASLt's default heuristic.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export BH_GEMM_TABLE=gpurun_out/tunableop_gfx950.csv
PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 900 python bench.py --gemm-table tune --steps 2 --warmup 2 \
  > gpurun_out/tune.log 2>&1 || { echo "tune rc=$?"; tail -20 gpurun_out/tune.log; exit 3; }
tail -3 gpurun_out/tune.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/tuned_bench.log 2>&1 && tail -1 gpurun_out/tuned_bench.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --gemm-table off > gpurun_out/default_bench.log 2>&1 && tail -1 gpurun_out/default_bench.log

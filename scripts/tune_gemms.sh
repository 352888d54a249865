#!/bin/bash
# Offline GEMM solution search (utils/gemm_tuning.py): time every hipBLASLt / rocBLAS solution of each
# library GEMM signature of the ResNet-50 bench step and the GPT-2 / BERT benchmark steps, merged into
# gpurun_out/tunableop_gfx950.csv (starting from the shipped table), then A/B each benchmark with the
# new table against hipBLASLt's default heuristic. Copy the table to beforeholiday_amd/utils/tuned/.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export BH_GEMM_TABLE=gpurun_out/tunableop_gfx950.csv
cp beforeholiday_amd/utils/tuned/tunableop_gfx950.csv "$BH_GEMM_TABLE" 2>/dev/null
what=${1:-all}
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; tail -1 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -20 "gpurun_out/$name.log"; exit 3; }
}
if [ "$what" = all ] || [ "$what" = resnet ]; then
  PYTORCH_TUNABLEOP_VERBOSE=1 run tune_r50 900 python bench.py --gemm-table tune --steps 2 --warmup 2
fi
if [ "$what" = all ] || [ "$what" = transformer ]; then
  PYTORCH_TUNABLEOP_VERBOSE=1 run tune_gpt 900 python benchmarks/bench_gpt.py --gemm-table tune --steps 2 --warmup 2
  PYTORCH_TUNABLEOP_VERBOSE=1 run tune_bert 900 python benchmarks/bench_bert.py --gemm-table tune --steps 2 --warmup 2
  run gpt_tuned 300 python benchmarks/bench_gpt.py --steps 10 --warmup 3
  run gpt_default 300 python benchmarks/bench_gpt.py --steps 10 --warmup 3 --gemm-table off
  run bert_tuned 300 python benchmarks/bench_bert.py --steps 10 --warmup 3
  run bert_default 300 python benchmarks/bench_bert.py --steps 10 --warmup 3 --gemm-table off
fi
if [ "$what" = all ] || [ "$what" = resnet ]; then
  run r50_tuned 300 python bench.py --steps 20 --warmup 5
  run r50_default 300 python bench.py --steps 20 --warmup 5 --gemm-table off
fi

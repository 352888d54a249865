#!/bin/bash
# sweep the reduction geometry (channel vectors per workgroup) x workgroup target x rows per lane
mkdir -p gpurun_out
run() { env "$@" timeout -k 10 90 python benchmarks/bench_bn.py > gpurun_out/bn_last.log 2>&1 || { echo "rc=$? $*"; exit 1; }; tail -1 gpurun_out/bn_last.log >> gpurun_out/bn_sweep2.jsonl; tail -1 gpurun_out/bn_last.log; }
run BH_BN_RED_CVB=256 BH_BN_STAT_BLOCKS=1024 BH_BN_RED_BLOCKS=256 BH_BN_RED_ROWS=32
cp gpurun_out/bn_last.log gpurun_out/bn_base_layers.log
for cvb in 8 16 32; do
  for blk in 512 1024 2048; do
    for rows in 8 16; do
      run BH_BN_RED_CVB=$cvb BH_BN_STAT_BLOCKS=$blk BH_BN_RED_BLOCKS=$blk BH_BN_RED_ROWS=$rows
    done
  done
done

#!/bin/bash
# after the wider finalize kernels: BN tests, then workgroup targets for stats / backward reduce
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_syncbn.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tsync.log 2>&1 || { tail -20 gpurun_out/tsync.log; exit 1; }
tail -1 gpurun_out/tsync.log
run() { env "$@" timeout -k 10 90 python benchmarks/bench_bn.py > gpurun_out/bn_last.log 2>&1 || { echo "rc=$? $*"; exit 1; }; tail -1 gpurun_out/bn_last.log | tee -a gpurun_out/bn_sweep3.jsonl; }
run X=1
for sb in 1024 2048 4096; do run BH_BN_STAT_BLOCKS=$sb BH_BN_STAT_ROWS=8; done
for rb in 512 1024 2048; do
  for cvb in 256 16; do run BH_BN_RED_BLOCKS=$rb BH_BN_RED_CVB=$cvb BH_BN_RED_ROWS=16; done
done

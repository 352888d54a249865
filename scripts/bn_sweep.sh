#!/bin/bash
# sweep BN reduction launch knobs with the BN microbenchmark (one process per setting)
for rb in 256 512 1024 2048; do
  for rr in 16 32 64 128; do
    BH_BN_RED_BLOCKS=$rb BH_BN_RED_ROWS=$rr timeout -k 10 60 python benchmarks/bench_bn.py | tail -1 || exit $?
  done
done

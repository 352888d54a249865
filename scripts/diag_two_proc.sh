#!/bin/bash
# two concurrent processes run benchmarks/diag_determinism.py on the one GPU; compare their per-op checksums
mkdir -p gpurun_out
DIAG_REPS=${DIAG_REPS:-3} DIAG_BWD=${DIAG_BWD:-0} DIAG_POISON=${DIAG_POISON:-} DIAG_BATCH=${DIAG_BATCH:-32} DIAG_PRE=0 DIAG_DUMP=gpurun_out/diag_a.txt timeout -k 10 150 python benchmarks/diag_determinism.py > gpurun_out/diag_a.log 2>&1 &
pa=$!
DIAG_REPS=${DIAG_REPS:-3} DIAG_BWD=${DIAG_BWD:-0} DIAG_POISON=${DIAG_POISON:-} DIAG_BATCH=${DIAG_BATCH:-32} DIAG_PRE=1 DIAG_DUMP=gpurun_out/diag_b.txt timeout -k 10 150 python benchmarks/diag_determinism.py > gpurun_out/diag_b.log 2>&1 &
pb=$!
wait $pa; ra=$?
wait $pb; rb=$?
echo "rc $ra $rb"
grep -v amdgpu gpurun_out/diag_a.log | grep -v "^ops" | sort | uniq -c | sort -rn | head -8; grep -v amdgpu gpurun_out/diag_b.log | grep -v "^ops" | sort | uniq -c | sort -rn | head -8
diff gpurun_out/diag_a.txt gpurun_out/diag_b.txt | head -20
exit 0

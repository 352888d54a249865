#!/bin/bash
# rocprofv3 counter passes over the ping-pong GEMM alone (plain 4096^3 bf16), then the summary
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_pp
i=0
for counters in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
                "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  echo "=== pass $i: $counters"
  timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmc_pp/p$i -o run -- \
      python3 benchmarks/pmc_kernels.py --only gemm_plain --iters 10 > gpurun_out/pmc_pp/p$i.log 2>&1
  rc=$?
  tail -2 gpurun_out/pmc_pp/p$i.log
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc, stopping"; exit $rc; fi
done
python3 scripts/pmc_summary.py gpurun_out/pmc_pp > gpurun_out/pmc_pp/summary.md
cat gpurun_out/pmc_pp/summary.md

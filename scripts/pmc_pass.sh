#!/bin/bash
# rocprofv3 counter passes over benchmarks/pmc_kernels.py, each pass in its own short run
# (one SQ/TCC group per pass, within the per-block hardware limits), then a per-kernel summary.
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for counters in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
                "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  echo "=== pass $i: $counters"
  timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmc/p$i -o run -- \
      python3 benchmarks/pmc_kernels.py --iters 10 > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  tail -2 gpurun_out/pmc/p$i.log
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc, stopping"; exit $rc; fi
done
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.md
cat gpurun_out/pmc/summary.md

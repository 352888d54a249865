#!/bin/bash
# rocprofv3 counter passes over the 3x3 conv weight-gradient kernel (benchmarks/bench_conv_wgrad.py, ONLY_R=3)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcw
i=0
for counters in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
                "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" \
                "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  echo "=== pass $i: $counters"
  timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmcw/p$i -o run -- \
      python3 benchmarks/bench_conv_wgrad.py > gpurun_out/pmcw/p$i.log 2>&1
  rc=$?
  tail -2 gpurun_out/pmcw/p$i.log
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc, stopping"; exit $rc; fi
done
python3 scripts/pmc_summary.py gpurun_out/pmcw > gpurun_out/pmcw/summary.md
cat gpurun_out/pmcw/summary.md

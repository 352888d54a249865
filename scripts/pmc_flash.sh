#!/bin/bash
# rocprofv3 counter passes over benchmarks/pmc_flash.py (flash attention); args go to pmc_flash.py
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcf
i=0
for counters in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
                "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM"; do
  i=$((i+1))
  echo "=== pass $i: $counters"
  timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmcf/p$i -o run -- \
      python3 benchmarks/pmc_flash.py "$@" > gpurun_out/pmcf/p$i.log 2>&1
  rc=$?
  tail -2 gpurun_out/pmcf/p$i.log
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc, stopping"; exit $rc; fi
done
python3 scripts/pmc_summary.py gpurun_out/pmcf > gpurun_out/pmcf/summary.md
cat gpurun_out/pmcf/summary.md

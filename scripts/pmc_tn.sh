#!/bin/bash
# rocprofv3 counter passes over the TN weight-gradient GEMM at the transformer shapes (benchmarks/pmc_tn.py)
export TMPDIR=/tmp
rm -rf gpurun_out/pmctn; mkdir -p gpurun_out/pmctn
i=0
for counters in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU" \
                "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
                "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  echo "=== pass $i: $counters"
  timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmctn/p$i -o run -- \
      python3 benchmarks/pmc_tn.py > gpurun_out/pmctn/p$i.log 2>&1
  rc=$?
  tail -1 gpurun_out/pmctn/p$i.log
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc, stopping"; exit $rc; fi
done
python3 scripts/pmc_summary.py gpurun_out/pmctn --table > gpurun_out/pmctn_table.md
python3 scripts/pmc_summary.py gpurun_out/pmctn > gpurun_out/pmctn_summary.md
rm -rf gpurun_out/pmctn/p*/
cat gpurun_out/pmctn_table.md

#!/bin/bash
# rocprofv3 counter passes over the ResNet-50 headline step (eager, 3 steps): per-kernel MFMA utilisation,
# VALU per MFMA, LDS bank conflicts, L2 hit rate for the conv / GEMM kernels (scripts/pmc_summary.py)
export TMPDIR=/tmp
rm -rf gpurun_out/pmcr; mkdir -p gpurun_out/pmcr
i=0
for counters in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU" \
                "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
                "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  echo "=== pass $i: $counters"
  timeout -s KILL 240 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmcr/p$i -o run -- \
      python3 bench.py --steps 3 --warmup 3 --graph off > gpurun_out/pmcr/p$i.log 2>&1
  rc=$?
  tail -1 gpurun_out/pmcr/p$i.log | cut -c1-200
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc, stopping"; exit $rc; fi
done
python3 scripts/pmc_summary.py gpurun_out/pmcr > gpurun_out/pmcr_summary.md
python3 scripts/pmc_summary.py gpurun_out/pmcr --table > gpurun_out/pmcr_table.md
rm -rf gpurun_out/pmcr/p*/
head -5 gpurun_out/pmcr_summary.md

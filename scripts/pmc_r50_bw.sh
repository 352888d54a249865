#!/bin/bash
# HBM traffic per kernel of the ResNet-50 bench step: one FETCH_SIZE pass, one WRITE_SIZE pass
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_bw
i=0
for counters in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "=== pass $i: $counters"
  timeout -s KILL 240 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmc_bw/p$i -o run -- \
      python3 bench.py --steps 2 --warmup 1 > gpurun_out/pmc_bw/p$i.log 2>&1
  rc=$?
  tail -2 gpurun_out/pmc_bw/p$i.log
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc, stopping"; exit $rc; fi
done
python3 scripts/pmc_bw_summary.py gpurun_out/pmc_bw --top 40 > gpurun_out/pmc_bw/summary.md
find gpurun_out/pmc_bw -name "*.csv" -size +20M -delete
cat gpurun_out/pmc_bw/summary.md

#!/bin/bash
# BERT-large whole-step capture with device dropout seeds: GPU suite, then eager vs captured A/B, then a
# kernel summary of the captured step
export TMPDIR=/tmp
SKIP_BENCH=1 bash scripts/gpu_full.sh
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2; do for g in off auto; do
  timeout -k 10 300 python benchmarks/bench_bert.py --steps 10 --warmup 3 --graph $g > gpurun_out/bert_g${g}_$r.log 2>&1 || exit $?
  echo "graph=$g $(grep -h 'bench_bert\]' gpurun_out/bert_g${g}_$r.log | cut -c1-160) $(tail -1 gpurun_out/bert_g${g}_$r.log | cut -c1-120)"
done; done
bash scripts/prof_bert.sh || exit $?
echo "bert summary: $(head -3 gpurun_out/bert_summary.md | tail -1)"
exit $rc

#!/bin/bash
# final round-6 validation: GPU suite, smoke, ResNet bench (scripts/gpu_r6_validate.sh), then the transformer
# benches with their capture check
export TMPDIR=/tmp
bash scripts/gpu_r6_validate.sh
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python benchmarks/bench_gpt.py --steps 10 --warmup 3 > gpurun_out/gpt_final.log 2>&1 || exit $?
echo "gpt: $(grep -h 'bench_gpt\]' gpurun_out/gpt_final.log | cut -c1-200) $(tail -1 gpurun_out/gpt_final.log | cut -c1-120)"
timeout -k 10 300 python benchmarks/bench_bert.py --steps 10 --warmup 3 > gpurun_out/bert_final.log 2>&1 || exit $?
echo "bert: $(grep -h 'bench_bert\]' gpurun_out/bert_final.log | cut -c1-200) $(tail -1 gpurun_out/bert_final.log | cut -c1-120)"
exit $rc

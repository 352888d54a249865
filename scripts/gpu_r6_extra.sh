#!/bin/bash
# round-6 extras: GPT-2 kernel summary (captured step), ResNet-50 O4 + FusedAdam (BASELINE configs[1])
export TMPDIR=/tmp
bash scripts/prof_gpt.sh || exit $?
echo "gpt summary: $(head -3 gpurun_out/gpt_summary.md | tail -1)"
timeout -k 10 300 python bench.py --opt-level O4 --optimizer adam --steps 20 --warmup 5 > gpurun_out/bench_o4.log 2>&1 || exit $?
echo "O4: $(tail -1 gpurun_out/bench_o4.log | cut -c1-160)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_o2b.log 2>&1 || exit $?
echo "O2: $(tail -1 gpurun_out/bench_o2b.log | cut -c1-160)"

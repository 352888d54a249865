# GPT-2-medium bench + kernel summary
bash scripts/gpu_steps.sh \
 "gpt:300:python benchmarks/bench_gpt.py --batch 8 --steps 10 --warmup 3" \
 "prof_gpt:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt -o run -- python benchmarks/bench_gpt.py --batch 8 --steps 5 --warmup 3 && python scripts/prof_summary.py gpurun_out/prof_gpt k_adam 3 gpurun_out/gpt_summary.md && rm -rf gpurun_out/prof_gpt"

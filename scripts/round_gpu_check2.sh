bash scripts/gpu_steps.sh \
 "bench_gemm1x1:300:python bench.py --steps 30 --warmup 10 --conv1x1 gemm" \
 "gpt_tp1:400:python benchmarks/bench_gpt.py --batch 8 --steps 10 --warmup 3" \
 "bert:400:python benchmarks/bench_bert.py --batch 16 --steps 10 --warmup 3"

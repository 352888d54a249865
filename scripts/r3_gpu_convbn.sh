# conv_bn kernel: numerics vs fp32 torch, then the per-shape microbenchmark
bash scripts/gpu_steps.sh \
 "t_convbn:300:python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_bn.py -m gpu" \
 "b_convbn:300:python benchmarks/bench_conv_bn.py --out gpurun_out/conv_bn_vs_unfused.jsonl"

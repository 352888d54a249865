# gemm_n64 kernel: GPU tests, kernel bench, same-box ResNet-50 A/B vs hipBLASLt (BH_GEMM_N64=0)
bash scripts/gpu_steps.sh \
 "tn64:240:python -u -m pytest tests/test_conv3x3.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'gemm_n64 or conv1x1 or module'" \
 "bn64:240:python benchmarks/bench_gemm_n64.py" \
 "warm:300:python bench.py --steps 5 --warmup 3" \
 "on1:300:python bench.py --steps 30 --warmup 5" \
 "off1:300:BH_GEMM_N64=0 python bench.py --steps 30 --warmup 5" \
 "on2:300:python bench.py --steps 30 --warmup 5" \
 "off2:300:BH_GEMM_N64=0 python bench.py --steps 30 --warmup 5"

# direct 3x3 conv kernel: numerics + timing vs MIOpen + ResNet-50 bench A/B on one box
bash scripts/gpu_steps.sh \
 "tconv:300:python -u -m pytest tests/test_conv3x3.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "bconv:300:python benchmarks/bench_conv3x3.py" \
 "r50_auto:300:python bench.py --steps 20 --warmup 5" \
 "r50_miopen:300:python bench.py --steps 20 --warmup 5 --conv3x3 miopen"

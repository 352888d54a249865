bash scripts/gpu_steps.sh \
 "twgrad:240:python -u -m pytest tests/test_conv3x3.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k wgrad" \
 "bwgrad:240:python benchmarks/bench_conv_wgrad.py"

# 3x3 conv: wide (1 WG/CU) vs streamed variant: numerics + timing
bash scripts/gpu_steps.sh \
 "tconv:300:python -u -m pytest tests/test_conv3x3.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "bconv2:300:python benchmarks/bench_conv3x3.py" \
 "bconv1:300:BH_CONV3X3_KERNEL=1 python benchmarks/bench_conv3x3.py" \
 "tconv1:300:BH_CONV3X3_KERNEL=1 python -u -m pytest tests/test_conv3x3.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider"

# same-box A/B: downsample 1x1/stride-2 weight gradient on the in-place MFMA kernel (default) vs
# MIOpen (BH_CONV1X1_S2=0)
bash scripts/gpu_steps.sh \
 "tconv:240:python -u -m pytest tests/test_conv3x3.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "bwg:240:ONLY_S2=1 python benchmarks/bench_conv_wgrad.py" \
 "warm:300:python bench.py --steps 5 --warmup 3" \
 "s2on1:300:python bench.py --steps 30 --warmup 5" \
 "s2off1:300:BH_CONV1X1_S2=0 python bench.py --steps 30 --warmup 5" \
 "s2on2:300:python bench.py --steps 30 --warmup 5" \
 "s2off2:300:BH_CONV1X1_S2=0 python bench.py --steps 30 --warmup 5"

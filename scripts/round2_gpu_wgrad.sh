# conv weight-gradient kernel: numerics, per-shape timing vs MIOpen; then the full re-validation
bash scripts/gpu_steps.sh \
 "twgrad:240:python -u -m pytest tests/test_conv3x3.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "bwgrad:240:python benchmarks/bench_conv_wgrad.py" \
 "bench_auto:400:python bench.py --steps 20 --warmup 5" \
 "gputests:900:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "rccl2:90:python scripts/rccl_same_gpu_probe.py"

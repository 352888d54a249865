# Fresh-container re-validation: full GPU suite, smoke, headline bench, and the RCCL same-GPU probe
bash scripts/gpu_steps.sh \
 "gputests:900:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:400:python bench.py --steps 20 --warmup 5" \
 "rccl2:90:python scripts/rccl_same_gpu_probe.py"

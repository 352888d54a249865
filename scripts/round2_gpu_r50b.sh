# residual-gradient fold + BN stats geometry: GPU tests, host-overhead probe, bench, BN microbench, profile
bash scripts/gpu_steps.sh \
 "tsync:300:python -u -m pytest tests/test_syncbn.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "host:300:python benchmarks/probe_host_overhead.py" \
 "bench:300:python bench.py --steps 20 --warmup 5" \
 "bn:200:python benchmarks/bench_bn.py" \
 "prof:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python bench.py --steps 8 --warmup 5 && python scripts/prof_summary.py gpurun_out/prof_r50 k_lamb2 3 gpurun_out/r50_summary.md"

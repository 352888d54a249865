bash scripts/gpu_steps.sh \
 "diag:200:python scripts/diag/fold_grads.py" \
 "t_convbn:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_bn.py -m gpu" \
 "b_convbn:300:python benchmarks/bench_conv_bn.py --out gpurun_out/conv_bn_vs_unfused.jsonl" \
 "bench_fold:400:python bench.py --steps 20 --warmup 5" \
 "prof:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python bench.py --steps 8 --warmup 5 && python scripts/prof_summary.py gpurun_out/prof_r50 k_lamb2 3 gpurun_out/r50_fold_summary.md && rm -rf gpurun_out/prof_r50"

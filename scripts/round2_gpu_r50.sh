# ResNet-50 bench A/B of the 1x1 conv paths + kernel summary of the default (auto) path.
bash scripts/gpu_steps.sh \
 "t1x1:300:python -u -m pytest tests/test_syncbn.py -m gpu -q -k conv1x1 --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "bench_auto:300:python bench.py --steps 20 --warmup 5 --conv1x1 auto" \
 "bench_miopen:300:python bench.py --steps 20 --warmup 5 --conv1x1 miopen" \
 "prof:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python bench.py --steps 8 --warmup 5 && python scripts/prof_summary.py gpurun_out/prof_r50 k_lamb2 3 gpurun_out/r50_summary.md"

# Round-3 baseline on a fresh box: cold-start trace of warmup step 1, bench, kernel profile.
bash scripts/gpu_steps.sh \
 "bench:400:python bench.py --steps 20 --warmup 5 --trace-warmup gpurun_out/warmup1_cprofile.txt" \
 "prof:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python bench.py --steps 8 --warmup 5 && python scripts/prof_summary.py gpurun_out/prof_r50 k_lamb2 3 gpurun_out/r50_summary.md && rm -rf gpurun_out/prof_r50"

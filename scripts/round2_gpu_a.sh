# Round 2, first GPU pass: full GPU suite, smoke (headline path in miniature; 3 runs, exit status
# checked each time), 1-GPU bench, self-spawned 2-rank bench (gloo rehearsal on one GPU), rocprofv3
# kernel summary of the bench.
bash scripts/gpu_steps.sh \
 "gputests:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "smoke:180:python -c 'import __graft_entry__ as g; g.smoke()' && python -c 'import __graft_entry__ as g; g.smoke()' && python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:300:python bench.py --steps 20 --warmup 5" \
 "spawn2:300:python bench.py --gpus 2 --steps 3 --warmup 2 --backend gloo --batch 32" \
 "prof:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python bench.py --steps 8 --warmup 5 && python scripts/prof_summary.py gpurun_out/prof_r50 k_lamb2 3 gpurun_out/r50_summary.md"

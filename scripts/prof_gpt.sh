# rocprofv3 kernel summary of the GPT-2-medium bench (3 steps after the FusedAdam marker)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/prof_gpt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt -o run -- python benchmarks/bench_gpt.py --steps 5 --warmup 2 > gpurun_out/prof_gpt.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_gpt "${PROF_MARKER:-k_adam}" 3 gpurun_out/gpt_summary.md
rc=$?
rm -rf gpurun_out/prof_gpt
exit $rc

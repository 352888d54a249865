# rocprofv3 kernel summary of the BERT-large bench (3 steps after the LAMB marker)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/prof_bert
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run -- python benchmarks/bench_bert.py --steps 5 --warmup 2 > gpurun_out/prof_bert.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_bert k_lamb2 3 gpurun_out/bert_summary.md
rc=$?
rm -rf gpurun_out/prof_bert
exit $rc

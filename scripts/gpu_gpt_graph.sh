#!/bin/bash
# GPT-2 capture after training_state learned the param-group device tensors
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_graph_checked.py tests/test_graph_rng.py > gpurun_out/t_gg.log 2>&1
rc=$?; tail -2 gpurun_out/t_gg.log; [ $rc -ne 0 ] && exit $rc
for g in auto off; do
  timeout -k 10 300 python benchmarks/bench_gpt.py --steps 10 --warmup 3 --graph $g > gpurun_out/gpt_g$g.log 2>&1 || exit $?
  echo "graph=$g $(grep -h 'bench_gpt\]' gpurun_out/gpt_g$g.log | cut -c1-200) $(tail -1 gpurun_out/gpt_g$g.log | cut -c1-110)"
done

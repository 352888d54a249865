#!/bin/bash
# row-pipelined fused LayerNorm backward vs the two-pass backward (Config.ln_bwd_fused) on BERT-large; GPT-2
# capture check
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_layer_norm.py tests/test_transformer_models.py tests/test_config.py tests/test_graph_rng.py > gpurun_out/t_ln.log 2>&1
rc=$?; tail -2 gpurun_out/t_ln.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python benchmarks/bench_ln_bwd.py > gpurun_out/ln_bwd_bench.log 2>&1 || exit $?; grep rep gpurun_out/ln_bwd_bench.log
for r in 1 2; do for f in 1 0; do
  BH_LN_BWD_FUSED=$f timeout -k 10 300 python benchmarks/bench_bert.py --steps 10 --warmup 3 > gpurun_out/bert_ln${f}_$r.log 2>&1 || exit $?
  echo "ln_fused=$f $(tail -1 gpurun_out/bert_ln${f}_$r.log | cut -c1-110)"
done; done
timeout -k 10 300 python benchmarks/bench_gpt.py --steps 10 --warmup 3 > gpurun_out/gpt_graph.log 2>&1 || exit $?
echo "gpt: $(grep -h 'bench_gpt\]' gpurun_out/gpt_graph.log | cut -c1-150) $(tail -1 gpurun_out/gpt_graph.log | cut -c1-120)"

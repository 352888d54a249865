bash scripts/gpu_steps.sh \
 "ce_test:300:python -u -m pytest tests/test_transformer_models.py tests/test_softmax.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "gpt_ce:300:python benchmarks/bench_gpt.py --batch 8 --steps 10 --warmup 3" \
 "bert_ce:300:python benchmarks/bench_bert.py --batch 16 --steps 10 --warmup 3"

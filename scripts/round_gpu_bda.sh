bash scripts/gpu_steps.sh \
 "bda_test:300:python -u -m pytest tests/test_dense.py tests/test_transformer_models.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "gpt_bda:300:python benchmarks/bench_gpt.py --batch 8 --steps 10 --warmup 3" \
 "bert_bda:300:python benchmarks/bench_bert.py --batch 16 --steps 10 --warmup 3"

# flash attention 32x32 backward: numerics + throughput vs the 16x16 kernels
bash scripts/gpu_steps.sh \
 "tflash:300:python -u -m pytest tests/test_fused_attention.py -m gpu -q -k flash --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "bwd32:300:python benchmarks/bench_flash.py --shapes gpt,bert,long --no-sdpa --tag bwd32" \
 "bwd16:300:BH_FLASH_BWD16=1 python benchmarks/bench_flash.py --shapes gpt,bert --no-sdpa --tag bwd16" \
 "tmodels:300:python -u -m pytest tests/test_transformer_models.py -m gpu -q -k flash --timeout 120 --timeout-method thread -p no:cacheprovider"

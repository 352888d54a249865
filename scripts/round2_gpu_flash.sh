# flash attention 32x32 forward variants (BH_FLASH_VAR): numerics + throughput
bash scripts/gpu_steps.sh \
 "tflash:300:python -u -m pytest tests/test_fused_attention.py -m gpu -q -k flash --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "var0:300:BH_FLASH_VAR=0 python benchmarks/bench_flash.py --shapes gpt,bert,long --no-sdpa --tag var0" \
 "var1:300:BH_FLASH_VAR=1 python benchmarks/bench_flash.py --shapes gpt,bert,long --no-sdpa --tag var1" \
 "var2:300:BH_FLASH_VAR=2 python benchmarks/bench_flash.py --shapes gpt,bert,long --no-sdpa --tag var2" \
 "tflash2:300:BH_FLASH_VAR=2 python -u -m pytest tests/test_fused_attention.py -m gpu -q -k flash --timeout 120 --timeout-method thread -p no:cacheprovider"

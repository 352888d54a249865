# direct 3x3 conv kernel: numerics, ResNet-50 bench A/B (auto vs MIOpen) and kernel summary
bash scripts/gpu_steps.sh \
 "tconv:300:python -u -m pytest tests/test_conv3x3.py tests/test_syncbn.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "r50_auto:300:python bench.py --steps 20 --warmup 5" \
 "r50_miopen:300:python bench.py --steps 20 --warmup 5 --conv3x3 miopen" \
 "r50_direct:300:python bench.py --steps 20 --warmup 5 --conv3x3 direct"

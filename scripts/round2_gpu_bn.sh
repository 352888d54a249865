# BN streaming kernels with deeper load pipelines: tests, per-shape floor, ResNet-50 bench
bash scripts/gpu_steps.sh \
 "tbn:300:python -u -m pytest tests/test_syncbn.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "floor:200:python benchmarks/bench_bn_floor.py" \
 "r50:300:python bench.py --steps 20 --warmup 5"

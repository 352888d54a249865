bash scripts/gpu_steps.sh \
 "sp_tests:300:python -u -m pytest tests/test_dense.py tests/test_transformer_models.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "gpt_tp2_sp_gloo:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29615 benchmarks/bench_gpt.py --tp 2 --sp --backend gloo --batch 2 --seq 512 --layers 4 --steps 2 --warmup 1" \
 "gpt_tp1:300:python benchmarks/bench_gpt.py --batch 8 --steps 10 --warmup 3"

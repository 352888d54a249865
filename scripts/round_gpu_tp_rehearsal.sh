bash scripts/gpu_steps.sh \
 "gpt_tp2_sp_gloo:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 benchmarks/bench_gpt.py --tp 2 --sp --backend gloo --batch 2 --seq 512 --layers 4 --steps 2 --warmup 1" \
 "gpt_tp2_gloo:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 benchmarks/bench_gpt.py --tp 2 --backend gloo --batch 2 --seq 512 --layers 4 --steps 2 --warmup 1" \
 "gpt_tp1_dp2_gloo:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29614 benchmarks/bench_gpt.py --tp 1 --backend gloo --batch 2 --seq 512 --layers 4 --steps 2 --warmup 1"

bash scripts/gpu_steps.sh \
 "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "smoke:180:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:300:python bench.py" \
 "gloo2:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 2 --backend gloo --batch 32"

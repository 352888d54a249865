#!/bin/bash
# world > 1 rehearsal of the headline bench on ONE GPU: two ranks over gloo share the card (the driver's
# multi-GPU runs use RCCL, one GPU per rank); checks the eager multi-rank path end to end
export TMPDIR=/tmp
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29613 bench.py --gpus 2 --backend gloo --steps 5 --warmup 3 > gpurun_out/rehearse2.log 2>&1
rc=$?; tail -2 gpurun_out/rehearse2.log | cut -c1-400; exit $rc

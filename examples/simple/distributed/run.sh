#!/bin/bash
# 2 ranks on this node (RCCL over xGMI); rendezvous on 127.0.0.1
python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NGPU:-2} --master-addr 127.0.0.1 \
  --master-port ${PORT:-29512} "$(dirname "$0")/distributed_data_parallel.py" "$@"

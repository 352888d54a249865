#!/bin/bash
# L1 cross-product (reference: tests/L1/common/run_test.sh): ResNet training under every
# opt level x loss-scale x keep-batchnorm setting, once with the fused extension path (--has-ext)
# and once with the python-only path, then an exact per-iteration loss comparison.
#   tests/L1/run_test.sh single_gpu [DATA_DIR]      # one process
#   tests/L1/run_test.sh distributed [DATA_DIR]     # 2 ranks (torchrun, RCCL)
set -e
MODE=${1:-single_gpu}
DATA=${2:-}
HERE=$(cd "$(dirname "$0")" && pwd)
MAIN="$HERE/../../examples/imagenet/main_amp.py"
OUT=${L1_OUT:-/tmp/bh_l1}
ARCH=${L1_ARCH:-resnet50}
COMMON="-a $ARCH --b ${L1_BATCH:-128} --deterministic --prints-to-process 5 --out-dir $OUT --quiet"
if [ "$MODE" == "distributed" ]; then
  RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 $MAIN"
else
  RUN="python $MAIN"
fi
rm -rf "$OUT" && mkdir -p "$OUT"
keep_bns=("" "--keep-batchnorm-fp32 True" "--keep-batchnorm-fp32 False")
loss_scales=("" "--loss-scale 1.0" "--loss-scale 128.0" "--loss-scale dynamic")
opt_levels=(O0 O1 O2 O3)
for ext in "--has-ext" ""; do
  for o in "${opt_levels[@]}"; do
    for ls in "${loss_scales[@]}"; do
      for kb in "${keep_bns[@]}"; do
        if [ "$o" == "O1" ] && [ -n "$kb" ]; then continue; fi
        echo "== $o $ls $kb $ext"
        $RUN $COMMON --opt-level $o $ls $kb $ext $DATA
      done
    done
  done
done
for o in "${opt_levels[@]}"; do
  for ls in "${loss_scales[@]}"; do
    for kb in "${keep_bns[@]}"; do
      if [ "$o" == "O1" ] && [ -n "$kb" ]; then continue; fi
      python "$HERE/compare.py" --dir "$OUT" --opt-level $o $ls $kb
    done
  done
done
echo "L1 cross-product: all trajectories identical"

#!/bin/bash
# round-6 check: conv / LN kernels vs fp32, conv microbench, ResNet headline, BERT step
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv3x3.py \
    tests/test_conv_bn.py tests/test_resnet_fold.py tests/test_layer_norm.py tests/test_transformer_models.py \
    tests/test_determinism.py > gpurun_out/t_v6.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/t_v6.log | head -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python benchmarks/bench_conv3x3.py > gpurun_out/conv_v6.log 2>&1 || exit $?
tail -1 gpurun_out/conv_v6.log
timeout -k 10 300 python bench.py > gpurun_out/bench_v6.log 2>&1 || exit $?
tail -1 gpurun_out/bench_v6.log | cut -c1-200
timeout -k 10 300 python benchmarks/bench_bert.py > gpurun_out/bert_v6.log 2>&1 || exit $?
tail -1 gpurun_out/bert_v6.log | cut -c1-200
BH_LN_RESID=0 timeout -k 10 300 python benchmarks/bench_bert.py > gpurun_out/bert_v6_noresid.log 2>&1 || exit $?
tail -1 gpurun_out/bert_v6_noresid.log | cut -c1-200

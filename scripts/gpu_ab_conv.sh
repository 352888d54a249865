#!/bin/bash
# conv-kernel correctness + microbench + headline bench in one GPU call (round 6 vmcnt work)
export TMPDIR=/tmp
export BH_FOLD_ERR_LOG=gpurun_out/fold_errs.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_conv3x3.py tests/test_conv_s2.py tests/test_conv_bn.py tests/test_dense.py tests/test_resnet_fold.py \
    tests/test_bn_fold.py tests/test_layer_norm.py tests/test_transformer_models.py tests/test_graph_checked.py > gpurun_out/t_conv.log 2>&1
rc=$?; tail -4 gpurun_out/t_conv.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python benchmarks/bench_conv3x3.py > gpurun_out/conv_v3.log 2>&1 || exit $?
tail -1 gpurun_out/conv_v3.log
timeout -k 10 200 python benchmarks/bench_conv_s2.py > gpurun_out/convs2_v3.log 2>&1 || exit $?
tail -2 gpurun_out/convs2_v3.log
timeout -k 10 300 python bench.py > gpurun_out/bench_v3.log 2>&1 || exit $?
tail -1 gpurun_out/bench_v3.log

#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv3x3.py \
    tests/test_conv_bn.py tests/test_resnet_fold.py tests/test_layer_norm.py \
    tests/test_transformer_models.py > gpurun_out/t_gc.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/t_gc.log | head -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_graph_checked.py > gpurun_out/t_gc2.log 2>&1
rc=$?; grep -E "passed|failed|eager_repeatable" gpurun_out/t_gc2.log | cut -c1-600 | head -6; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python benchmarks/bench_conv3x3.py > gpurun_out/conv_v4.log 2>&1 || exit $?
tail -1 gpurun_out/conv_v4.log
for on in 0 1; do BH_CONV3X3_BWD_EPI=$on timeout -k 10 300 python bench.py --steps 20 --warmup 6 > gpurun_out/bench_epi$on.log 2>&1 || exit $?; echo "bwd_epi=$on $(tail -1 gpurun_out/bench_epi$on.log | cut -c1-120)"; done
bash scripts/prof_resnet.sh || exit $?
head -60 gpurun_out/resnet_summary.md | tail -52 | cut -c1-160
bash scripts/pmc_resnet.sh

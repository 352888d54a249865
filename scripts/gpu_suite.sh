#!/bin/bash
# Parametrised GPU driver: bash scripts/gpu_suite.sh <preset> [<preset> ...]
# Each preset expands to named steps run by gpu_steps.sh (own time limit each, stop at the first crash).
#   tests   : pytest -m gpu (whole suite, one process)
#   fold    : BN-folded conv kernels + block numerics
#   micro   : conv_bn microbenchmark (strip / tiled GEMM vs hipBLASLt + BatchNorm passes)
#   bench   : bench.py 1 GPU (20 steps), with a cProfile of warmup step 1
#   prof    : rocprofv3 kernel trace of the bench + per-kernel summary (gpurun_out/r50_summary.md)
#   nofold  : bench.py with BH_FOLD_BN=0 (A/B)
#   graph   : bench.py with the whole step replayed as a HIP graph
#   peer    : IPC peer memory + SyncBN GPU tests
#   tune    : offline hipBLASLt / rocBLAS solution search -> gpurun_out/tunableop_gfx950.csv
steps=()
for preset in "$@"; do
  case "$preset" in
    tests) steps+=("tests:900:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu") ;;
    fold) steps+=("fold:400:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_bn.py tests/test_resnet_fold.py tests/test_ddp.py -m gpu") ;;
    micro) steps+=("micro:300:python benchmarks/bench_conv_bn.py --out gpurun_out/conv_bn_vs_unfused.jsonl") ;;
    bench) steps+=("bench:400:python bench.py --steps 20 --warmup 5 --trace-warmup gpurun_out/warmup1_cprofile.txt") ;;
    graphtest) steps+=("graphtest:300:python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_graphs.py -m gpu") ;;
    graphdiff) steps+=("graphdiff:300:python scripts/diag/graph_diff.py") ;;
    graph) steps+=("graph:400:python bench.py --steps 20 --warmup 5 --graph on") ;;
    nofold) steps+=("nofold:400:BH_FOLD_BN=0 python bench.py --steps 20 --warmup 5") ;;
    prof) steps+=("prof:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python bench.py --steps 8 --warmup 5 && python scripts/prof_summary.py gpurun_out/prof_r50 k_lamb2 3 gpurun_out/r50_summary.md && rm -rf gpurun_out/prof_r50") ;;
    peer) steps+=("peer:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_peer_memory.py tests/test_syncbn.py -m gpu") ;;
    tune) steps+=("tune:900:BH_GEMM_TABLE=gpurun_out/tunableop_gfx950.csv PYTORCH_TUNABLEOP_VERBOSE=1 python bench.py --gemm-table tune --steps 2 --warmup 2") ;;
    cbr) steps+=("cbr:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_bias_relu.py tests/test_contrib_basic.py -m gpu") ;;
    conv3) steps+=("conv3:300:python benchmarks/bench_conv3x3.py") ;;
    gpt) steps+=("gpt:400:python benchmarks/bench_gpt.py --batch 8 --steps 10 --warmup 3") ;;
    gptprof) steps+=("gptprof:400:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt -o run -- python benchmarks/bench_gpt.py --batch 8 --steps 6 --warmup 3 && python scripts/prof_summary.py gpurun_out/prof_gpt k_adam 3 gpurun_out/gpt_summary.md && rm -rf gpurun_out/prof_gpt") ;;
    *) echo "unknown preset $preset"; exit 2 ;;
  esac
done
bash scripts/gpu_steps.sh "${steps[@]}"

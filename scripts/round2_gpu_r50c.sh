# ResNet-50 kernel summary with the direct 3x3 conv (auto) + counters of the conv kernel
bash scripts/gpu_steps.sh \
 "tconv:200:python -u -m pytest tests/test_conv3x3.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "prof:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python bench.py --steps 8 --warmup 5 && python scripts/prof_summary.py gpurun_out/prof_r50 k_lamb2 3 gpurun_out/r50_summary.md && rm -rf gpurun_out/prof_r50" \
 "pmc:200:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_conv -o run -- python3 benchmarks/bench_conv3x3.py"

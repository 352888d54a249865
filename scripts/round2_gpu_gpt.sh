# dense dispatch autotune: tests, GPT-2-medium bench (tuned vs all-hipBLASLt), kernel summary
bash scripts/gpu_steps.sh \
 "tdense:300:python -u -m pytest tests/test_dense.py tests/test_gemm_mfma.py tests/test_transformer_models.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "gpt:300:python benchmarks/bench_gpt.py --batch 8 --steps 10 --warmup 3" \
 "gpt_lib:300:BH_DENSE_MFMA=0 python benchmarks/bench_gpt.py --batch 8 --steps 10 --warmup 3" \
 "prof_gpt:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt -o run -- python benchmarks/bench_gpt.py --batch 8 --steps 5 --warmup 3 && python scripts/prof_summary.py gpurun_out/prof_gpt k_adam 3 gpurun_out/gpt_summary.md && rm -rf gpurun_out/prof_gpt"

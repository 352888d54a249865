# ResNet-50 bench under MIOpen solver-selection knobs (wrw split-K zero-fill avoidance)
bash scripts/gpu_steps.sh \
 "base:300:python bench.py --steps 20 --warmup 5" \
 "nowrwgtc:300:MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 python bench.py --steps 20 --warmup 5" \
 "noatomic:300:MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_PK_ATOMIC_ADD_FP16=0 python bench.py --steps 20 --warmup 5"

#!/bin/bash
# A/B the MIOpen solver families used by the ResNet-50 bench (immediate mode): each variant
# disables one family so MIOpen's heuristic falls back to the next-best solver.
mkdir -p gpurun_out
run() {
  name=$1; shift
  echo "=== $name: $*" | tee -a gpurun_out/miopen_sweep.log
  env "$@" timeout -k 10 240 python bench.py --steps 15 --warmup 5 2>>gpurun_out/miopen_sweep.err | tee -a gpurun_out/miopen_sweep.log
  rc=${PIPESTATUS[0]}
  if [ $rc -ne 0 ]; then echo "rc=$rc, stopping"; exit $rc; fi
}
run base X=1
run no_asm_wrw MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0
run no_asm_fwd MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0
run no_asm_bwd MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0

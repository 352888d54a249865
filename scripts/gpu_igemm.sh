#!/bin/bash
# LDS-staged stride-2 implicit GEMM (Config.igemm_lds): tests, then interleaved kernel + ResNet bench A/B
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv_s2.py tests/test_config.py > gpurun_out/t_igemm.log 2>&1
rc=$?; tail -3 gpurun_out/t_igemm.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in 1 0; do
  BH_IGEMM_LDS=$v timeout -k 10 200 python benchmarks/bench_conv_s2.py > gpurun_out/s2_${v}_$r.log 2>&1 || exit $?
  echo "lds=$v r=$r $(python3 -c "import json,sys; print(' '.join(f\"{d['C']}/{d['dir']}={d['own_ms']}\" for d in map(json.loads, (l for l in open(sys.argv[1]) if l.startswith('{'))) if d['dir'] in ('fwd','fwd_pro_stats','dgrad')))" gpurun_out/s2_${v}_$r.log)"
done; done
for r in 1 2; do for v in 1 0; do
  BH_IGEMM_LDS=$v timeout -k 10 300 python bench.py --steps 30 --warmup 8 > gpurun_out/rn_lds${v}_$r.log 2>&1 || exit $?
  echo "lds=$v $(tail -1 gpurun_out/rn_lds${v}_$r.log | cut -c1-100)"
done; done

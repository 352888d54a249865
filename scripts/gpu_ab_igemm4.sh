#!/bin/bash
# stride-2 igemm epilogue stores through a buffer resource vs 64-bit global stores
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv_s2.py tests/test_resnet_fold.py > gpurun_out/t_wgp.log 2>&1
rc=$?; tail -2 gpurun_out/t_wgp.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_so.sh "python benchmarks/bench_conv_s2.py" ig4s2 || exit $?
bash scripts/ab_so.sh "python bench.py --steps 30 --warmup 8" ig4rn || exit $?
for f in gpurun_out/ig4s2_*.log; do echo "$f $(python3 -c "import json,sys; print(' '.join(f\"{d['C']}/{d['dir']}={d['own_ms']}\" for d in map(json.loads, (l for l in open(sys.argv[1]) if l.startswith('{'))) if d['dir'] in ('fwd_pro_stats','dgrad')))" $f)"; done
for f in gpurun_out/ig4rn_*.log; do echo "$f $(tail -1 $f | cut -c1-100)"; done

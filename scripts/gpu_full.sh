#!/bin/bash
# GPU validation run (bash scripts/gpu_full.sh) used with gpurun: the gpu-marked suite (no first-failure stop), then one 1-GPU
# bench. Stops before the bench when pytest ended by a signal / time limit (a fault or hang).
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
    ${PYTEST_ARGS:-} > gpurun_out/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
brc=$?
tail -2 gpurun_out/bench.log
exit $brc

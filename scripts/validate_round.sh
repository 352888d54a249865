#!/bin/bash
# Round-end validation on one GPU (used with gpurun): the gpu-marked suite, smoke(), then bench.py twice.
# Writes gpurun_out/validation.txt; stops before the benches when pytest ended by a signal / time limit.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/validation.txt
: > $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest -m gpu rc=$rc: $(tail -1 gpurun_out/pytest.log)" | tee -a $out
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?
echo "smoke rc=$src: $(tail -1 gpurun_out/smoke.log)" | tee -a $out
if [ $src -ne 0 ]; then exit $src; fi
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench$i.log 2>&1 || exit $?
  echo "bench $i: $(tail -1 gpurun_out/bench$i.log)" | tee -a $out
done
exit $rc

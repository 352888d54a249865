#!/bin/bash
# the two-process IPC capture test with and without deferred plan uploads, verbose, stacks dumped on timeout
export TMPDIR=/tmp
BH_GRAPH_DEFER_UPLOADS=0 timeout -k 10 170 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_graph_checked.py -k ipc > gpurun_out/ipc0.log 2>&1
rc=$?; echo "defer=0 rc=$rc"; tail -3 gpurun_out/ipc0.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 170 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_graph_checked.py -k ipc > gpurun_out/ipc1.log 2>&1
rc=$?; echo "defer=1 rc=$rc"; tail -3 gpurun_out/ipc1.log
exit $rc

#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_graph_checked.py > gpurun_out/t_gc.log 2>&1
grep -E "passed|failed|mismatch" gpurun_out/t_gc.log | head -4
bash scripts/prof_resnet.sh || exit $?
head -60 gpurun_out/resnet_summary.md | tail -52 | cut -c1-160
bash scripts/pmc_resnet.sh

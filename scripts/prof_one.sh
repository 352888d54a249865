#!/bin/bash
# rocprofv3 kernel-trace --stats of one python command; per-kernel totals over the whole run go to
# gpurun_out/<name>_summary.md (scripts/prof_summary.py). usage: prof_one.sh <name> <python args...>
name=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf "gpurun_out/prof_$name"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$name" -o run -- python "$@" > "gpurun_out/prof_$name.log" 2>&1
rc=$?
python scripts/prof_summary.py "gpurun_out/prof_$name" "^no-marker$" 1 "gpurun_out/${name}_summary.md" || rc=$?
rm -rf "gpurun_out/prof_$name"
exit $rc

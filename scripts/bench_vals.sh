#!/bin/bash
# print "name img/s ms" for gpurun_out/<name>.log bench logs
for f in "$@"; do
  l=$(grep -h '"metric"' "gpurun_out/$f.log" 2>/dev/null | tail -1)
  if [ -n "$l" ]; then echo "$f $(echo "$l" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; else echo "$f -"; fi
done

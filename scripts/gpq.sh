#!/bin/bash
# usage: scripts/gpq.sh OUTFILE TIMEOUT 'command'   -- retries only while gpurun reports no free slot (exit 3)
out=$1; to=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $out; then echo "rc=$rc" >> $out; exit 0; fi
  sleep 150
done

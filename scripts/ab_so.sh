#!/bin/bash
# same-box A/B of two builds of the extension: runs CMD with the tree's _C (new), then with ab/_C_base.so
# swapped in, alternating twice. usage: ab_so.sh "<cmd>" name
cmd=$1; name=$2
so=$(ls beforeholiday_amd/_C*.so)
cp "$so" /tmp/_C_new.so
for r in 1 2; do
  cp /tmp/_C_new.so "$so"; timeout -k 10 300 bash -c "$cmd" > "gpurun_out/${name}_new$r.log" 2>&1 || exit $?
  cp ab/_C_base.so "$so"; timeout -k 10 300 bash -c "$cmd" > "gpurun_out/${name}_base$r.log" 2>&1 || exit $?
done
cp /tmp/_C_new.so "$so"

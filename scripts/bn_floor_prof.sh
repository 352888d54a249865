# kernel-level times of the BN passes at one small and one mid ResNet-50 layer shape
export TMPDIR=/tmp
for shp in 14x256 7x512 28x512; do
  BN_SHAPE=$shp timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bnprof_$shp -o run -- python3 benchmarks/bench_bn_floor.py > gpurun_out/bnprof_$shp.log 2>&1 || exit 1
  f=$(find gpurun_out/bnprof_$shp -name "*kernel_stats.csv" | head -1)
  echo "== $shp"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print('%-70s calls=%5s avg_us=%8.2f' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))
"
done

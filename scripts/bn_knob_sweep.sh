# rocprofv3 kernel-time sweep of the BN reduction geometry knobs over bench_bn.py (all ResNet-50 shapes)
export TMPDIR=/tmp
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bnsw_$tag -o run -- python3 benchmarks/bench_bn.py > gpurun_out/bnsw_$tag.log 2>&1 || return 1
  f=$(find gpurun_out/bnsw_$tag -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$tag" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = {}
for r in rows:
    n = r['Name']
    for key in ('k_stats_nhwc', 'k_stats_finalize', 'k_bwd_reduce_nhwc', 'k_bwd_reduce_finalize', 'k_fwd_nhwc', 'k_dgrad_nhwc'):
        if key in n:
            tot[key] = tot.get(key, 0.0) + float(r['TotalDurationNs']) / 1e6
print(sys.argv[2], {k: round(v, 2) for k, v in sorted(tot.items())})
PY
  rm -rf gpurun_out/bnsw_$tag
}
run base BH_BN_DUMMY=1 && \
run srows4 BH_BN_STAT_ROWS=4 && \
run srows8 BH_BN_STAT_ROWS=8 && \
run rrows8 BH_BN_RED_ROWS=8 && \
run rrows16 BH_BN_RED_ROWS=16 && \
run rblk1024 BH_BN_RED_BLOCKS=1024 BH_BN_RED_ROWS=8 && \
run ewrows4 BH_BN_EW_ROWS=4 && \
run ewblk4096 BH_BN_EW_BLOCKS=4096

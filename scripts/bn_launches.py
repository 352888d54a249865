"""Per-launch durations of the BN kernels in one training step of a rocprofv3 database, with the
workgroup grid (identifies the layer shape). Usage: python scripts/bn_launches.py <dir> [pattern]"""
import glob
import re
import sqlite3
import sys


def main():
    db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_stats_nhwc|k_bwd_reduce_nhwc|k_fwd_nhwc|k_dgrad_nhwc|finalize")
    cur = sqlite3.connect(db).cursor()
    rows = cur.execute("select d.start, d.end, s.kernel_name, d.grid_size_x, d.grid_size_y, d.workgroup_size_x "
                       "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
                       "order by d.start").fetchall()
    marks = [i for i, r in enumerate(rows) if "k_lamb2" in r[2]]
    a, b = marks[-2], marks[-1]
    step = rows[a + 1:b + 1]
    agg = {}
    for st, en, name, gx, gy, wx in step:
        if not pat.search(name):
            continue
        short = re.search(r"(k_\w+?)(I|E|<|$)", name)
        short = short.group(1) if short else name[:40]
        key = (short, gx // max(wx, 1), gy)
        agg.setdefault(key, []).append((en - st) / 1e3)
    tot = {}
    for (k, gx, gy), ds in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        tot[k] = tot.get(k, 0) + sum(ds)
        print(f"{k:28s} grid=({gx},{gy}) n={len(ds):3d} mean={sum(ds)/len(ds):7.1f} us  total={sum(ds):8.1f} us")
    print({k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()

"""Per-kernel HBM traffic from rocprofv3 FETCH_SIZE / WRITE_SIZE passes under <dir>/p*/ (kilobytes
per dispatch, as rocprofv3 derives them): launches, mean time, MB read / written per dispatch and the
effective bandwidth (read + write) / time, sorted by total time. Kernel names are shortened to the
identifier before the first template / argument list.

    python scripts/pmc_bw_summary.py gpurun_out/pmc_bw [--top 30]
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r"_ZN2bh12_GLOBAL__N_1\d+(k_\w+?)I", name) or re.search(r"bh::(k_\w+)", name)
    if m:
        return m.group(1)
    return re.split(r"[<(]", name)[0][:60]


def main():
    d = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 30
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r.get("Kernel_Name", "?"))
                c = r["Counter_Name"]
                vals[k][c].append(float(r["Counter_Value"]))
                vals[k]["dur_" + c].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for k, cs in vals.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        n = len(cs["FETCH_SIZE"])
        us = sum(cs["dur_FETCH_SIZE"]) / n
        rd = sum(cs["FETCH_SIZE"]) / n / 1024
        wr = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) / 1024
        rows.append((us * n, k, n, us, rd, wr, (rd + wr) / 1024 / (us / 1e6) / 1e3 if us else 0.0))
    rows.sort(reverse=True)
    print("| kernel | dispatches | mean us | MB read | MB written | effective TB/s |")
    print("|---|---|---|---|---|---|")
    for _, k, n, us, rd, wr, bw in rows[:top]:
        print(f"| `{k}` | {n} | {us:.1f} | {rd:.1f} | {wr:.1f} | {bw:.2f} |")


if __name__ == "__main__":
    main()

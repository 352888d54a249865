"""Summarise a rocprofv3 kernel trace for steady-state training steps.

Usage: python scripts/prof_summary.py <dir with *_kernel_trace.csv> <marker-regex> [steps] [out.md]

Steps are delimited by occurrences of a marker kernel (one launch per training step, e.g. the
optimizer's last kernel). The last ``steps`` complete intervals are aggregated by kernel name:
total / per-step time, share, launch count, and GPU-busy vs. wall span per step (a gap means the
GPU waited for the host). The big trace CSVs are deleted afterwards so gpurun_out stays small.
"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    d, marker = sys.argv[1], re.compile(sys.argv[2])
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(d, "summary.md")
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    # rocprofv3 >= ROCm 7 writes a rocpd SQLite database by default (``kernels`` view)
    for f in glob.glob(os.path.join(d, "**", "*_results.db"), recursive=True):
        import sqlite3

        con = sqlite3.connect(f)
        rows.extend((int(s), int(e), n) for s, e, n in con.execute("select start, end, name from kernels"))
        con.close()
    rows.sort()
    marks = [i for i, r in enumerate(rows) if marker.search(r[2])]
    lines = []
    if len(marks) < 2:
        lines.append(f"marker {marker.pattern!r} found {len(marks)} times; aggregating whole trace")
        lo, hi, n = 0, len(rows), 1
    else:
        use = marks[-(nsteps + 1):]
        lo, hi, n = use[0] + 1, use[-1] + 1, len(use) - 1
    seg = rows[lo:hi]
    agg = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for s, e, name in seg:
        short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))[:110]
        agg[short][0] += e - s
        agg[short][1] += 1
        busy += e - s
    span = (seg[-1][1] - seg[0][0]) if seg else 0
    lines.append(f"# kernel time per step (last {n} steps, marker {marker.pattern!r})\n")
    lines.append(f"wall span/step: {span / n / 1e6:.3f} ms; GPU busy/step (sum of kernel times): "
                 f"{busy / n / 1e6:.3f} ms; kernels/step: {len(seg) / n:.0f}\n")
    # idle gaps (GPU waiting on the host) in the last step: where they are tells a host sync at the
    # step boundary from host-issue-bound stretches of small kernels
    last = rows[marks[-2] + 1:marks[-1] + 1] if len(marks) >= 2 else seg
    gaps, end = [], None
    for s_, e_, name in last:
        if end is not None and s_ > end:
            gaps.append((s_ - end, prev, name))
        end = e_ if end is None else max(end, e_)
        prev = name
    short = lambda n_: re.sub(r"\(.*", "", n_.replace("(anonymous namespace)::", ""))[:60]
    tot_gap = sum(g[0] for g in gaps)
    lines.append(f"idle in the last step: {tot_gap / 1e6:.3f} ms in {len(gaps)} gaps; largest:\n")
    for g_, a_, b_ in sorted(gaps, reverse=True)[:8]:
        lines.append(f"* {g_ / 1e3:.1f} us after `{short(a_)}` before `{short(b_)}`")
    lines.append("")
    lines.append("| kernel | ms/step | share | launches/step |")
    lines.append("|---|---|---|---|")
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:150]:
        lines.append(f"| `{k}` | {t / n / 1e6:.3f} | {100.0 * t / max(busy, 1):.1f}% | {c / n:.1f} |")
    # per-launch durations (us) of the last step for the top kernels, in launch order
    last = rows[marks[-2] + 1: marks[-1] + 1] if len(marks) >= 2 else seg
    per = collections.defaultdict(list)
    for s_, e_, name in last:
        per[re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))[:110]].append(round((e_ - s_) / 1e3, 1))
    lines.append("\n## per-launch us (last step, launch order) for kernels > 0.5 ms/step (and PROF_LIST matches)\n")
    extra = re.compile(os.environ["PROF_LIST"]) if os.environ.get("PROF_LIST") else None
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        if t / n / 1e6 < 0.5 and not (extra and extra.search(k)):
            continue
        lines.append(f"* `{k[:60]}`: {per[k]}")
    # neighbours of library helper kernels (fills, copies) in the last step: which op launched them
    helpers = re.compile(os.environ.get("PROF_NEIGHBOURS", r"SubTensorOp|copyBuffer|fillBuffer"))
    pairs = collections.Counter()
    for i, (s_, e_, name) in enumerate(last):
        if helpers.search(name):
            before = short(last[i - 1][2]) if i > 0 else "-"
            after = short(last[i + 1][2]) if i + 1 < len(last) else "-"
            pairs[(short(name), before, after)] += 1
    if pairs:
        lines.append("\n## helper kernels in the last step: (kernel, launched after, launched before) x count\n")
        for (k, b_, a_), c in pairs.most_common(20):
            lines.append(f"* {c} x `{k}` after `{b_}` before `{a_}`")
    text = "\n".join(lines) + "\n"
    with open(out, "w") as fh:
        fh.write(text)
    print(text)
    for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
        if "kernel_stats" not in f:
            os.remove(f)


if __name__ == "__main__":
    main()

"""Per-kernel register / spill / occupancy / LDS table of one HIP source (hipcc -Rpass-analysis).
usage: python scripts/kernel_resources.py beforeholiday_amd/csrc/kernels/<file>.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                      "-Ibeforeholiday_amd/csrc/include", "-c", src, "-o", "/tmp/_kr.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt in r["name"]:
        print(f"{r.get('VGPRs','?'):>4} v {r.get('AGPRs','?'):>4} a spill {r.get('VGPRs Spill','?'):>4} "
              f"occ {r.get('Occupancy [waves/SIMD]','?')} lds {r.get('LDS Size [bytes/block]','?'):>6}  {r['name'][:110]}")

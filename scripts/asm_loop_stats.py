"""Instruction histogram of a kernel's depth-1 loop body from a hipcc --save-temps .s file.

    python scripts/asm_loop_stats.py attn-hip-amdgcn-amd-amdhsa-gfx950.s k_flash_fwd32 [--all]

Matches every function whose mangled name contains the given substring; a basic block belongs to
the loop when its label line carries hipcc's "Loop: Header=... Depth=1" note (the header itself or
"in Loop: Header=..."). Prints the instruction count, the VALU count (v_* except MFMA) and the most
common opcodes: the quick way to see what a source change did to the per-iteration work.
"""
import re
import sys
from collections import Counter


def functions(text, pat):
    for m in re.finditer(r"^(_Z[^:\s]+):", text, re.M):
        name = m.group(1)
        if pat in name:
            end = text.find(".Lfunc_end", m.end())
            yield name, text[m.end():end]


def loop_blocks(body):
    blocks, cur, inloop = [], [], False
    for line in body.split("\n"):
        if re.match(r"^(\.LBB\S+:|; %bb\.\d+:)", line):
            if inloop:
                blocks.append(cur)
            cur = []
            inloop = "Depth=1" in line
            continue
        if ("Loop Header: Depth=1" in line or "Loop: Header=" in line and "Depth=1" in line) and not cur:
            inloop = True
            continue
        s = line.strip()
        if s and not s.startswith((".", ";")):
            cur.append(s)
    if inloop:
        blocks.append(cur)
    return [i for b in blocks for i in b]


def main():
    path, pat = sys.argv[1], sys.argv[2]
    text = open(path).read()
    for name, body in functions(text, pat):
        ins = loop_blocks(body)
        c = Counter(i.split()[0] for i in ins)
        valu = sum(v for k, v in c.items() if k.startswith("v_") and "mfma" not in k)
        mfma = sum(v for k, v in c.items() if "mfma" in k)
        print(f"{name}\n  loop instrs {len(ins)}  valu {valu}  mfma {mfma}")
        print("  " + ", ".join(f"{k} {v}" for k, v in c.most_common(30 if "--all" in sys.argv else 16)))


if __name__ == "__main__":
    main()

"""Average rocprofv3 counter values per kernel over all passes under <dir>/p*/ and print a table
(MFMA busy share, LDS bank-conflict share, L2 hit rate where the counters are present)."""
import collections
import csv
import glob
import os
import re
import sys


def main():
    d = sys.argv[1]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "?")
                if "k_gemm_tn" in name:
                    # template <T, PART, AK>: PART = split-K partials, AK = the NN (A row-major) layout
                    part = "Lb1E" in name.split("k_gemm_tn")[1][:12]
                    name = "gemm_tn<" + ("split" if part else "unsplit") + ">"
                elif "k_tn_reduce" in name:
                    name = "tn_reduce"
                elif "k_gemm_pp" in name:
                    name = "gemm_pp<256x256>"
                elif "gemm_nt" in name:
                    big = "Li8ELi4E" in name or "Cfg<2, 4, 8, 4, 2>" in name
                    name = "gemm_nt<" + ("256x256" if big else "128x128") + ">"
                elif "k_flash_fwd" in name:
                    name = "flash_fwd"
                elif "k_flash_bwd_dq" in name or "k_flash_dq32" in name:
                    name = "flash_bwd_dq"
                elif "k_flash_bwd_dkdv" in name or "k_flash_dkdv32" in name:
                    name = "flash_bwd_dkdv"
                elif "attn_fwd" in name:
                    name = "attn_fwd"
                elif "attn_bwd" in name:
                    name = "attn_bwd"
                elif "k_conv3x3" in name:
                    # the first template bool after the dtype is FLIP (the data gradient)
                    kind = "dgrad" if re.search(r"k_conv3x3I(DF16_|DF16b)Lb1E", name) else "fwd"
                    # G is the first int template argument (the weight-buffer count NB also is an int)
                    gm = re.search(r"k_conv3x3I(?:DF16_|DF16b)Lb[01]ELi(\d)E", name)
                    g = "G" + (gm.group(1) if gm else "?")
                    name = f"conv3x3_{kind}<{g}>"
                elif "k_conv_wgrad" in name:
                    geo = {"Li3ELi14ELi2E": "3x3 56x56", "Li3ELi7ELi4E": "3x3 28x28", "Li3ELi4ELi7E": "3x3 14x14",
                           "Li3ELi2ELi7E": "3x3 7x7", "Li1ELi28ELi1E": "1x1"}
                    name = "conv_wgrad<" + next((v for k, v in geo.items() if k in name), "?") + ">"
                elif "k_igemm" in name:
                    name = "igemm<s2 3x3 " + ("dgrad" if "Lb0ELb0E" in name or "Lb0ELb1E" in name else "fwd") + ">"
                elif "k_c1x1" in name:
                    name = "c1x1<strip 1x1>"
                elif "k_gemm_n64" in name:
                    name = "gemm_n64<1x1 K=64>"
                elif "k_stem" in name:
                    name = "stem<" + ("wgrad" if "wgrad" in name else "fwd") + ">"
                else:
                    continue
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
                vals[name]["duration_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    if "--table" in sys.argv:  # one row per kernel family: the derived ratios only
        print("| kernel | dispatches | us / dispatch | MFMA util | non-MFMA VALU / MFMA | LDS conflict share | "
              "L2 hit | wait share of wave cycles |")
        print("|---|---|---|---|---|---|---|---|")
        for k in sorted(vals):
            m = {c: sum(v) / len(v) for c, v in vals[k].items()}
            n = len(vals[k]["duration_us"]) // max(1, len([c for c in vals[k] if c != "duration_us"]))

            def f(x):
                return "-" if x is None else f"{x:.2f}"
            util = (m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
                    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE") else None)
            valu = ((m["SQ_INSTS_VALU"] - m["SQ_INSTS_MFMA"]) / m["SQ_INSTS_MFMA"]
                    if m.get("SQ_INSTS_MFMA") and "SQ_INSTS_VALU" in m else None)
            lds = (m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
                   if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE") else None)
            l2 = (m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
                  if "TCC_HIT_sum" in m and (m["TCC_HIT_sum"] + m.get("TCC_MISS_sum", 0)) else None)
            wait = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"] if m.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in m else None
            print(f"| {k} | {n} | {m['duration_us']:.1f} | {f(util)} | {f(valu)} | {f(lds)} | {f(l2)} | {f(wait)} |")
        return
    print("| kernel | counter | mean per dispatch |")
    print("|---|---|---|")
    for k in sorted(vals):
        m = {c: sum(v) / len(v) for c, v in vals[k].items()}
        for c in sorted(m):
            print(f"| {k} | {c} | {m[c]:.4g} |")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m and m["SQ_BUSY_CYCLES"]:
            print(f"| {k} | MFMA busy / SQ busy | {m['SQ_VALU_MFMA_BUSY_CYCLES'] / m['SQ_BUSY_CYCLES']:.3f} |")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
            # per-SIMD share of the GPU-active cycles (GRBM_GUI_ACTIVE summed over 8 XCDs, 1024 SIMDs)
            util = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
            print(f"| {k} | MFMA utilisation (busy / (GUI_ACTIVE/8 x 1024 SIMDs)) | {util:.3f} |")
        if m.get("SQ_INSTS_MFMA") and "SQ_INSTS_VALU" in m:
            # (SQ_INSTS_VALU counts the MFMAs too)
            print(f"| {k} | non-MFMA VALU per MFMA | {(m['SQ_INSTS_VALU'] - m['SQ_INSTS_MFMA']) / m['SQ_INSTS_MFMA']:.2f} |")
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            print(f"| {k} | LDS bank-conflict cycles / LDS active | {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.3f} |")
        if "TCC_HIT_sum" in m and (m["TCC_HIT_sum"] + m.get("TCC_MISS_sum", 0)):
            print(f"| {k} | L2 hit rate | {m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.3f} |")


if __name__ == "__main__":
    main()

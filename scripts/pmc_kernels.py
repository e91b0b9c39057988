"""Mean of every collected PMC counter per kernel over the dispatches of several rocprofv3 --pmc
passes (each pass a directory with run_counter_collection.csv), plus derived shares.

usage: python scripts/pmc_kernels.py <title> <pass dir> [<pass dir> ...] > profiles/X.md
"""
import collections
import csv
import os
import re
import sys


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", name)[:80]


def main():
    title, dirs = sys.argv[1], sys.argv[2:]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        names, dur = {}, {}
        for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
            i = int(r["Dispatch_Id"])
            names[i] = short(r["Kernel_Name"])
            dur[i] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            per[i][r["Counter_Name"]] += float(r["Counter_Value"])
        for i, cs in per.items():
            agg[names[i]]["duration_us"].append(dur[i] / 1e3)
            for c, v in cs.items():
                agg[names[i]][c].append(v)
    print(f"# {title}\n")
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"## `{k}` ({len(cs['duration_us'])} dispatch-passes)\n")
        print("| counter | mean per dispatch |\n|---|---|")
        for c in sorted(m):
            print(f"| {c} | {m[c]:.4g} |")
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            wc = m["SQ_WAVE_CYCLES"]
            sh = {c: m[c] / wc for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if c in m}
            print("\nshares of wave cycles: " + ", ".join(f"{c[3:]} {100 * v:.0f}%" for c, v in sh.items()))
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            us = m["duration_us"]
            print(f"\nMFMA busy / (duration x 2.4 GHz x 1024 SIMDs): "
                  f"{100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / (us * 1e-6 * 2.4e9 * 1024):.1f}%")
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            print(f"\nL2 hit rate: {100 * m['TCC_HIT_sum'] / max(1.0, m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.1f}%")
        print()


if __name__ == "__main__":
    main()

"""Per-kernel PMC summary of a whole training step (scripts/gpu/pmc_step.sh output).

usage: python scripts/pmc_summary.py <pmcstep dir> <title> > profiles/X.md

Pass p1 = FETCH_SIZE, p2 = WRITE_SIZE (TCC, KiB moved between L2 and memory), p3 = SQ counters +
GRBM_GUI_ACTIVE.  Per kernel (name truncated): dispatches, mean duration, HBM read/write bytes per
dispatch, achieved memory bandwidth, MFMA busy share of the dense peak
(SQ_VALU_MFMA_BUSY_CYCLES / (kernel time x 2.4 GHz x 1,024 SIMDs); calibrated on the hipBLASLt GEMMs,
whose 0.42-0.54 matches their measured 1.05-1.35 PFLOP/s of 2.5) and the LDS bank-conflict share.
GRBM_GUI_ACTIVE is kept in the raw data but not used: it sums the 8 XCDs' counters.
"""
import collections
import csv
import os
import re
import sys

N_CU = 256


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name[:70]


def load(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        disp[d] = (short(r["Kernel_Name"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    return disp, per


def main():
    root, title = sys.argv[1], sys.argv[2]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in ("p1", "p2", "p3"):
        disp, per = load(os.path.join(root, p, "run_counter_collection.csv"))
        for d, (k, ns) in disp.items():
            a = agg[k]
            if p == "p1":
                a["n"] += 1
                a["ns"] += ns
            if p == "p3":
                a["ns3"] += ns
            for c, v in per[d].items():
                a[c] += v
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["ns"])
    tot = sum(a["ns"] for _, a in rows)
    print(f"# {title}\n")
    print(__doc__.split("\n\n", 1)[1].strip() + "\n")
    print("| kernel | calls | mean us | % time | HBM read MB/call | HBM write MB/call | HBM TB/s | MFMA busy / peak | LDS conflict / LDS active |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k, a in rows:
        if a["ns"] < 0.002 * tot:
            continue
        n = max(a["n"], 1)
        rd = a["FETCH_SIZE"] * 1024 / n
        wr = a["WRITE_SIZE"] * 1024 / n
        us = a["ns"] / n / 1e3
        bw = (rd + wr) / (a["ns"] / n) / 1e3 if a["ns"] else 0.0
        mf = a["SQ_VALU_MFMA_BUSY_CYCLES"] / (a["ns3"] * 2.4 * N_CU * 4) if a["ns3"] else 0.0
        lds = a["SQ_LDS_BANK_CONFLICT"] / a["SQ_LDS_IDX_ACTIVE"] if a["SQ_LDS_IDX_ACTIVE"] else 0.0
        print(f"| `{k}` | {int(a['n'])} | {us:.1f} | {100 * a['ns'] / tot:.1f} | {rd / 1e6:.1f} | {wr / 1e6:.1f} | "
              f"{bw:.2f} | {100 * mf:.1f} % | {100 * lds:.1f} % |")


if __name__ == "__main__":
    main()

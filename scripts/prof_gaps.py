"""Idle time between kernels in a rocprofv3 kernel trace: per step (delimited by one kernel that runs once per
step, default the CE kernel), the step period, the union of kernel busy time and the largest gaps.

usage: python scripts/prof_gaps.py <run_kernel_trace.csv> [--marker ce_kernel] [--last 5]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="ce_kernel")
    ap.add_argument("--last", type=int, default=5)
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    for s in range(max(0, len(marks) - 1 - a.last), len(marks) - 1):
        seg = rows[marks[s]:marks[s + 1]]
        t0, t1 = seg[0][0], rows[marks[s + 1]][0]
        busy, cur_s, cur_e, gaps = 0, seg[0][0], seg[0][1], []
        prev_name = seg[0][2]
        for st, en, name in seg[1:]:
            if st > cur_e:
                busy += cur_e - cur_s
                gaps.append((st - cur_e, prev_name[:60], name[:60]))
                cur_s, cur_e = st, en
            else:
                cur_e = max(cur_e, en)
            prev_name = name
        busy += min(cur_e, t1) - cur_s
        period = t1 - t0
        gaps.sort(reverse=True)
        print(f"step {s}: period {period / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {100 * (1 - busy / period):.2f} %, "
              f"{len(seg)} kernels, {len(gaps)} gaps")
        for g, p, n in gaps[:a.top]:
            print(f"    {g / 1e3:8.1f} us  after {p}  before {n}")


if __name__ == "__main__":
    main()

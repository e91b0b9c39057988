"""Turn a rocprofv3 ``--kernel-trace --stats`` kernel_stats.csv into the markdown table kept
under profiles/ (per-step milliseconds, share, calls/step, average microseconds).

usage: python scripts/prof_summary.py <kernel_stats.csv> <steps> <title> [notes...] > profiles/X.md
"""
import csv
import sys


def main():
    path, steps, title = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    notes = sys.argv[4:]
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    for n in notes:
        print(n + "\n")
    print(f"Kernel time {tot / 1e6:.1f} ms over {steps} steps = {tot / 1e6 / steps:.2f} ms/step.\n")
    print("| ms/step | % | calls/step | avg us | kernel |")
    print("|---|---|---|---|---|")
    for r in rows:
        t = float(r["TotalDurationNs"])
        if t / tot < 0.0002:
            continue
        print(f"| {t / 1e6 / steps:.3f} | {100 * t / tot:.1f} | {int(r['Calls']) / steps:.1f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | `{r['Name'][:110]}` |")


if __name__ == "__main__":
    main()

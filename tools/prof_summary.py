"""Summarise a rocprofv3 kernel_stats.csv: top kernels and per-family totals.

usage: python tools/prof_summary.py gpurun_out/prof/bench_kernel_stats.csv [steps] [top]
"""
import csv
import re
import sys


def family(name):
    m = re.match(r"(?:void )?(?:tvq::)?([A-Za-z_0-9:]+)", name)
    return m.group(1) if m else name


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    calls = sum(int(r["Calls"]) for r in rows)
    print(f"total {tot / 1e6 / steps:.3f} ms/step, {calls / steps:.0f} launches/step")
    for r in rows[:top]:
        t = float(r["TotalDurationNs"])
        print(f"{t / tot * 100:5.1f}% {t / 1e6 / steps:7.3f}ms {int(r['Calls']) / steps:7.1f}x "
              f"{float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:100]}")
    fam = {}
    for r in rows:
        f = family(r["Name"])
        a = fam.setdefault(f, [0.0, 0])
        a[0] += float(r["TotalDurationNs"])
        a[1] += int(r["Calls"])
    print("--- families")
    for f, (t, c) in sorted(fam.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{t / tot * 100:5.1f}% {t / 1e6 / steps:7.3f}ms {c / steps:7.1f}x  {f}")


if __name__ == "__main__":
    main()

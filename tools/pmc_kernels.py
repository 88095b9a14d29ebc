"""Average PMC counters per kernel family of one rocprofv3 counter_collection.csv.
usage: python tools/pmc_kernels.py counter_collection.csv [name-filter]"""
import collections
import csv
import re
import sys


def main():
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    cs = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(sys.argv[1])):
        k = re.match(r"(?:void )?(?:tvq::)?([A-Za-z_0-9:]+)(<[^(]*>)?", r["Kernel_Name"])
        name = (k.group(1) + (k.group(2) or "")) if k else r["Kernel_Name"]
        if flt in name:
            cs[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, c in sorted(cs.items()):
        print(f"== {name[:90]}")
        for cn, v in sorted(c.items()):
            print(f"   {cn:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")


if __name__ == "__main__":
    main()

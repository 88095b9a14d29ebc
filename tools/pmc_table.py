"""Average PMC counters per tvq kernel from gpurun_out/pmc/p_* runs.
usage: python tools/pmc_table.py [dir]"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    cases = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "p_*", "run_counter_collection.csv"))):
        case = re.sub(r"_\d+$", "", os.path.basename(os.path.dirname(f)))
        for r in csv.DictReader(open(f)):
            if "tvq::" not in r["Kernel_Name"]:
                continue
            k = re.match(r"(?:void )?tvq::([a-z_]+)(<[^(]*>)?", r["Kernel_Name"])
            name = k.group(1) + (k.group(2) or "")
            cases[(case, name)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (case, name), cs in sorted(cases.items()):
        print(f"== {case} {name[:90]}")
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v) / len(v):14.0f}")


if __name__ == "__main__":
    main()

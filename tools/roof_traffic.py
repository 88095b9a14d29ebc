"""traffic_bytes per op for bench.py's roofline legs from the rocprofv3 --pmc passes of
tools/gpu_roofline.sh: per kernel name substring (an op may be several launches, e.g. the
weight-gradient GEMM + its slab sum), the average FETCH_SIZE (x2, the gfx950 correction of
MI355X_MICROARCH.md §HBM) + WRITE_SIZE per launch, summed over the op's kernels; plus the
per-launch SQ counters and the rocprofv3 average duration.
usage: python tools/roof_traffic.py DIR out.json "op description" substr [substr ...]"""
import collections
import csv
import glob
import json
import sys


def per_kernel(path, counters):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] in counters:
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def one(d, pattern):
    f = glob.glob(f"{d}/{pattern}/**/*counter_collection.csv", recursive=True)
    return f[0] if f else None


def main():
    d, out, desc, subs = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4:]
    fetch = per_kernel(one(d, "fetch"), {"FETCH_SIZE"})
    write = per_kernel(one(d, "write"), {"WRITE_SIZE"})
    sqf = one(d, "sq")
    sq = per_kernel(sqf, {"SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_MFMA", "SQ_WAVES",
                          "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS", "SQ_WAIT_ANY",
                          "SQ_WAVE_CYCLES"}) if sqf else {}
    stats = glob.glob(f"{d}/stats/**/*kernel_stats.csv", recursive=True)
    durs = {}
    if stats:
        for r in csv.DictReader(open(stats[0])):
            durs[r["Name"]] = float(r["AverageNs"]) / 1e3
    res = {"op": desc, "kernels": {}}
    fmb = wmb = us = 0.0
    for sub in subs:
        names = [k for k in fetch if sub in k]
        if not names:
            continue
        k = names[0]
        fk = sum(fetch[k]["FETCH_SIZE"]) / len(fetch[k]["FETCH_SIZE"]) * 2.0 / 1024  # KB -> MB
        wl = write.get(k, {}).get("WRITE_SIZE", [0.0])
        wk = sum(wl) / len(wl) / 1024
        dk = next((v for n, v in durs.items() if sub in n), None)
        q = {c: sum(v) / len(v) for c, v in sq.get(k, {}).items()}
        res["kernels"][sub] = {"fetch_MB": round(fk, 3), "write_MB": round(wk, 3),
                               "launches": len(fetch[k]["FETCH_SIZE"]),
                               "avg_us_rocprof": dk, "sq_per_launch": q}
        fmb += fk
        wmb += wk
        us += dk or 0.0
    res["fetch_MB"] = round(fmb, 3)
    res["write_MB"] = round(wmb, 3)
    res["traffic_bytes"] = int((fmb + wmb) * 1024 * 1024)
    res["op_avg_us_rocprof"] = round(us, 2)
    import os
    tf = os.path.join(os.path.dirname(os.path.abspath(__file__)), ".tree")
    res["tree"] = open(tf).read().strip() if os.path.exists(tf) else None  # git HEAD profiled
    res["source"] = ("tools/gpu_roofline.sh: rocprofv3 --kernel-trace --stats, then --pmc FETCH_SIZE / "
                     "WRITE_SIZE / SQ_* passes of tools/roofline_only.py; FETCH_SIZE doubled per "
                     "MI355X_MICROARCH.md HBM section; tools/roof_traffic.py")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

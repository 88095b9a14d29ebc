"""Step-only kernel table from a rocprofv3 kernel_trace.csv of `bench.py --no-sampler
--no-roofline --no-config0 --no-cpu-baseline` (graph-replayed joint steps).

The last `steps` steps are cut at the AdamW launches (2 per step: stage1, stage2) and
every kernel in them is tabulated: calls per step, average duration, time per step and
share of the summed kernel time.  Also reports the wall span per step (the critical path
of the concurrent streams) and launches per step.
usage: python tools/step_table.py trace.csv [steps] [out.csv] [start-marker kernel]"""
import collections
import csv
import re
import sys


def fam(n):
    m = re.match(r"(?:void )?(?:tvq::)?([A-Za-z_0-9:]+)(<[^(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    out = sys.argv[3] if len(sys.argv) > 3 else None
    marker = sys.argv[4] if len(sys.argv) > 4 else None
    if marker:  # the last `steps` units each START at a `marker` launch (one per unit) and
        # run to the end of the trace (tools/sampler_graph_prof.py: add_i64_kernel, the
        # seed advance that opens every replayed sampling batch)
        starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
        sel = rows[starts[-steps]:]
    else:
        # a step ends at its AdamW: one adamw2_kernel (both optimizers) or two adamw_kernel
        ends = [i for i, r in enumerate(rows) if "adamw2_kernel" in r["Kernel_Name"]]
        per = 1
        if not ends:
            ends = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
            per = 2
        first = ends[-1 - per * steps] + 1
        sel = rows[first:ends[-1] + 1]
    t0 = int(sel[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in sel)
    agg = collections.defaultdict(lambda: [0, 0])
    for r in sel:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[fam(r["Kernel_Name"])][0] += d
        agg[fam(r["Kernel_Name"])][1] += 1
    total = sum(v[0] for v in agg.values())
    print(f"{steps} steps: wall {(t1 - t0) / 1e3 / steps:.1f} us/step, {len(sel) / steps:.0f} launches/step, "
          f"summed kernel time {total / 1e3 / steps:.1f} us/step")
    table = sorted(agg.items(), key=lambda x: -x[1][0])
    w = csv.writer(open(out, "w")) if out else None
    if w:
        w.writerow(["kernel", "calls_per_step", "avg_us", "us_per_step", "pct_of_kernel_time"])
    for k, (d, c) in table:
        row = [k, round(c / steps, 2), round(d / c / 1e3, 2), round(d / steps / 1e3, 1),
               round(100 * d / total, 2)]
        if w:
            w.writerow(row)
    for row in table[:30]:
        k, (d, c) = row
        print(f"{d / steps / 1e3:9.1f} us/step {c / steps:6.1f}x {d / c / 1e3:8.2f} us  {k[:100]}")


if __name__ == "__main__":
    main()

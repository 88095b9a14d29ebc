"""Per-queue kernel sequence of the last unit of a rocprofv3 kernel_trace.csv that starts at a
marker kernel (tools/sampler_graph_prof.py: add_i64_kernel opens every replayed sampling
batch): start offset from the unit's first kernel, duration and name, per queue, and each
queue's busy time.  usage: python tools/batch_seq.py trace.csv marker [out.txt]"""
import collections
import csv
import re
import sys


def fam(n):
    m = re.match(r"(?:void )?(?:tvq::)?([A-Za-z_0-9:]+)(<[^(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"]]
    unit = rows[starts[-1]:]
    t0 = int(unit[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in unit)
    out = [f"unit: {len(unit)} kernels, wall {(t1 - t0) / 1e3:.1f} us"]
    q = collections.defaultdict(list)
    for r in unit:
        q[r["Queue_Id"]].append(r)
    for qid, rs in q.items():
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e3
        out.append(f"queue {qid}: {len(rs)} kernels, busy {busy:.1f} us")
        for r in rs:
            s = (int(r["Start_Timestamp"]) - t0) / 1e3
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            out.append(f"  {s:9.1f} {d:8.2f}  {fam(r['Kernel_Name'])}")
    text = "\n".join(out)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text + "\n")
    print("\n".join(out[:1] + [l for l in out if l.startswith("queue")]))


if __name__ == "__main__":
    main()

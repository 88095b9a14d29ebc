"""Critical-path view of one graph-replayed step from a rocprofv3 kernel_trace.csv.

The step's last kernels are its AdamW launches (`per_step` of them, one per optimizer; one
adamw2_kernel for both when the trace has it):
the last step is everything after the previous step's final AdamW through the last one.
Prints its wall span, per-queue busy time and kernel families ranked by time per queue.
usage: python tools/step_timeline.py trace.csv [per_step] [top] [seq_out]
seq_out: also write every queue's kernel sequence (start offset, duration, gap to the
previous kernel on that queue) to that file."""
import collections
import csv
import re
import sys


def fam(n):
    m = re.match(r"(?:void )?(?:tvq::)?([A-Za-z_0-9:]+)(<[^(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    ends = [i for i, r in enumerate(rows) if "adamw2_kernel" in r["Kernel_Name"]]
    if ends:  # one launch for both optimizers
        per = 1
    else:
        ends = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
    step = rows[ends[-1 - per] + 1:ends[-1] + 1]
    starts = ends[::per]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in step)
    print(f"last step: {len(step)} kernels, wall {(t1 - t0) / 1e3:.1f} us "
          f"({len(starts)} step starts found)")
    q = collections.defaultdict(list)
    for r in step:
        q[r["Queue_Id"]].append(r)
    for qid, rs in q.items():
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs)
        span = max(int(r["End_Timestamp"]) for r in rs) - int(rs[0]["Start_Timestamp"])
        print(f"queue {qid}: {len(rs)} kernels, busy {busy / 1e3:.1f} us, span {span / 1e3:.1f} us")
        f = collections.defaultdict(lambda: [0, 0])
        for r in rs:
            k = fam(r["Kernel_Name"])
            f[k][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            f[k][1] += 1
        for k, (d, c) in sorted(f.items(), key=lambda x: -x[1][0])[:top]:
            print(f"   {d / 1e3:8.1f} us {c:4d}x  {k[:110]}")
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            for qid, rs in q.items():
                f.write(f"queue {qid}\n")
                prev = None
                for r in rs:
                    s0, s1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                    gap = (s0 - prev) / 1e3 if prev is not None else 0.0
                    f.write(f"{(s0 - t0) / 1e3:9.1f} {(s1 - s0) / 1e3:7.2f} {gap:6.2f}  "
                            f"{fam(r['Kernel_Name'])[:100]}\n")
                    prev = s1


if __name__ == "__main__":
    main()

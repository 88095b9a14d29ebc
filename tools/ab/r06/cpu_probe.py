"""Probe the GPU box's host CPUs: affinity, cgroup quota, and one CPU-port joint step at a few
thread counts (progress to stdout per step)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count(), flush=True)
for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpuset.cpus.effective"):
    try:
        print(f, open(f).read().strip(), flush=True)
    except OSError as e:
        print(f, "n/a", e, flush=True)
print("env", {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "MAX_JOBS")}, flush=True)
from oracle import cpu_baseline  # noqa: E402
from oracle.cpu_baseline import cpu_model  # noqa: E402
print("cpu", cpu_model(), flush=True)
js = cpu_baseline.JointStep(B=256)
for n in [int(a) for a in sys.argv[1:]]:
    torch.set_num_threads(n)
    for i in range(3):
        t0 = time.perf_counter()
        js.step()
        print(f"threads {n} step {i}: {time.perf_counter() - t0:.3f} s", flush=True)

#!/bin/bash
# fused loss head: tests, then its kernel time in the step (rocprofv3 stats over a short bench)
set -o pipefail
mkdir -p gpurun_out/tlce
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tied_ce.py tests/test_fullsize_parity.py::test_stage2_per_prior_backward_roots_bitwise > gpurun_out/tlce/tests.log 2>&1 || { tail -20 gpurun_out/tlce/tests.log; exit 1; }
tail -1 gpurun_out/tlce/tests.log
rm -rf gpurun_out/tlce/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tlce/prof -o p -- python bench.py --steps 10 --warmup 2 --no-sampler --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs > gpurun_out/tlce/prof.log 2>&1 || { tail -5 gpurun_out/tlce/prof.log; exit 1; }
S=$(find gpurun_out/tlce/prof -name "*kernel_stats.csv" | head -1)
python - "$S" <<'PY'
import csv, sys
for r in csv.reader(open(sys.argv[1])):
    if "tlce" in r[0] or r[0] == "Name":
        print(r[0][:50], r[1], r[3], r[5], r[6])
PY
T=$(find gpurun_out/tlce/prof -name "*kernel_trace.csv" | head -1)
python - "$T" <<'PY'
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
gk = [k for k in rows[0] if "Grid" in k]
by = collections.defaultdict(list)
for r in rows:
    if "tlce_kernel" in r["Kernel_Name"]:
        by[tuple(r[k] for k in gk)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in by.items():
    print("tlce grid", k, "n", len(v), "avg us %.1f" % (sum(v) / len(v)))
PY
find gpurun_out/tlce/prof -name "*kernel_trace.csv" -delete
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-roofline --no-config0 --no-cpu-baseline --no-sampler > gpurun_out/tlce/bench.log 2>&1 || { tail -5 gpurun_out/tlce/bench.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/tlce/bench.log').read().strip().splitlines()[-1]);print('bench',d['ms_per_step'],d.get('stage1_ms_per_step'),d.get('stage2_ms_per_step'))"
done

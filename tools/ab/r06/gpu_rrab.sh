#!/bin/bash
# A/B of a library build (lib_ab/, base) against the in-tree build: per-kernel time of the
# step's named kernel under rocprofv3 (5 graph-replayed steps each), then the joint step alternated
set -o pipefail
mkdir -p gpurun_out/rrab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
K=${AB_KERNEL:-reduce_rows_batch4}
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs"
for n in base new; do
  if [ $n = base ]; then export TVQ_HIP_LIB=$GRAFT_REPO_ROOT/lib_ab/libtvq_hip.so; else unset TVQ_HIP_LIB; fi
  rm -rf gpurun_out/rrab/p$n
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rrab/p$n -o p -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/rrab/p$n.log 2>&1 || { tail -20 gpurun_out/rrab/p$n.log; exit 1; }
  T=$(find gpurun_out/rrab/p$n -name "*kernel_trace.csv" | head -1)
  python - "$T" "$K" $n <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        d[r["Queue_Id"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for q, v in sorted(d.items()):
    v = v[-10:]
    print(sys.argv[3], "queue", q, "n", len(v), "us", " ".join(f"{x:.1f}" for x in v))
PY
  rm -f "$T"
done
unset TVQ_HIP_LIB
show() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['ms_per_step'],d.get('stage1_ms_per_step'),d.get('stage2_ms_per_step'))"; }
for rep in 1 2; do
  for n in base new; do
    if [ $n = base ]; then export TVQ_HIP_LIB=$GRAFT_REPO_ROOT/lib_ab/libtvq_hip.so; else unset TVQ_HIP_LIB; fi
    timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-roofline --no-config0 --no-cpu-baseline --no-sampler > gpurun_out/rrab/b$n.log 2>&1 || { tail -5 gpurun_out/rrab/b$n.log; exit 1; }
    echo "$n $(show gpurun_out/rrab/b$n.log)"
  done
done

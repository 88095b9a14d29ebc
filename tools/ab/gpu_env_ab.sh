#!/bin/bash
# step bench under a list of environment settings (AB_CASES: ';'-separated "VAR=val VAR2=val")
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
IFS=';' read -ra CASES <<< "$AB_CASES"
for c in "${CASES[@]}"; do
  env $c timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  echo "[$c] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_ab.log)"
done

#!/bin/bash
# Kernel tables of one part of the joint step alone (graph-replayed): the LF band alone
# (TVQ_BENCH_ONLY=stage1 TVQ_BENCH_BANDS=LF) and stage2 alone (TVQ_BENCH_ONLY=stage2).
set -o pipefail
mkdir -p gpurun_out/chain
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs"
for part in lf s2; do
  if [ $part = lf ]; then export TVQ_BENCH_ONLY=stage1 TVQ_BENCH_BANDS=LF; else export TVQ_BENCH_ONLY=stage2; unset TVQ_BENCH_BANDS; fi
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/chain/$part.log 2>&1 || { tail -5 gpurun_out/chain/$part.log; exit 1; }
  echo "$part $(python -c "import json;print(json.loads(open('gpurun_out/chain/$part.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  rm -rf gpurun_out/chain/prof_$part
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/chain/prof_$part -o k -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/chain/prof_$part.log 2>&1 || { tail -5 gpurun_out/chain/prof_$part.log; exit 1; }
  T=$(find gpurun_out/chain/prof_$part -name "*kernel_trace.csv" | head -1)
  python tools/step_table.py "$T" 5 gpurun_out/chain/${part}_table.csv > gpurun_out/chain/${part}_table.txt
  head -1 gpurun_out/chain/${part}_table.txt
  rm -rf gpurun_out/chain/prof_$part
done

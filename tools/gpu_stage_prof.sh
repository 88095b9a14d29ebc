#!/bin/bash
# Kernel tables of each part of the joint step alone (TVQ_BENCH_ONLY / TVQ_BENCH_BANDS), so
# per-kernel times are not stretched by the other streams: stage2, stage1 LF band, HF band.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for part in stage2 LF HF; do
  rm -rf gpurun_out/prof_$part
  if [ $part = stage2 ]; then E="TVQ_BENCH_ONLY=stage2"; else E="TVQ_BENCH_ONLY=stage1 TVQ_BENCH_BANDS=$part"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$part -o p -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/prof_$part.log 2>&1 || { tail -20 gpurun_out/prof_$part.log; exit 1; }
  T=$(find gpurun_out/prof_$part -name "*kernel_trace.csv" | head -1)
  python tools/step_table.py "$T" 5 gpurun_out/table_$part.csv | head -3
done

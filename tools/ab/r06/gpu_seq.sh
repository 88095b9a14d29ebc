#!/bin/bash
# Per-queue kernel sequences (start, duration, gap) of one graph-replayed step: the joint step
# and the stage1 LF band alone (tools/step_timeline.py seq_out).
set -o pipefail
mkdir -p gpurun_out/r6s
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs"
for part in joint LF; do
  rm -rf gpurun_out/r6s/$part
  if [ $part = joint ]; then E="X=1"; else E="TVQ_BENCH_ONLY=stage1 TVQ_BENCH_BANDS=$part"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6s/$part -o p -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/r6s/$part.log 2>&1 || { tail -20 gpurun_out/r6s/$part.log; exit 1; }
  T=$(find gpurun_out/r6s/$part -name "*kernel_trace.csv" | head -1)
  python tools/step_timeline.py "$T" 2 12 gpurun_out/r6s/seq_$part.txt > gpurun_out/r6s/timeline_$part.txt
  head -1 gpurun_out/r6s/timeline_$part.txt
  rm -rf gpurun_out/r6s/$part
done

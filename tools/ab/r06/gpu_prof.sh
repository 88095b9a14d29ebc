#!/bin/bash
# Kernel tables: stage2 alone, then the joint step (rocprofv3 kernel trace, graph-replayed).
set -o pipefail
mkdir -p gpurun_out/r6p
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs"
for part in ${PARTS:-stage2 joint}; do
  rm -rf gpurun_out/r6p/$part
  if [ $part = joint ]; then E="X=1"; elif [ $part = stage2 ] || [ $part = stage1 ]; then E="TVQ_BENCH_ONLY=$part"; else E="TVQ_BENCH_ONLY=stage1 TVQ_BENCH_BANDS=$part"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6p/$part -o p -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/r6p/$part.log 2>&1 || { tail -20 gpurun_out/r6p/$part.log; exit 1; }
  T=$(find gpurun_out/r6p/$part -name "*kernel_trace.csv" | head -1)
  python tools/step_table.py "$T" 5 gpurun_out/r6p/table_$part.csv > gpurun_out/r6p/table_$part.txt
  head -3 gpurun_out/r6p/table_$part.txt
  python tools/step_timeline.py "$T" 2 12 > gpurun_out/r6p/timeline_$part.txt
  rm -f "$T"
done

#!/bin/bash
# Stage2 alone under the kernel trace: per-queue busy time / sequences and the kernel table
# (what bounds stage2_ms_per_step).  PART=S2 (default) or S1.
set -o pipefail
PART=${PART:-S2}
mkdir -p gpurun_out/r6s
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs"
if [ $PART = S2 ]; then ONLY=stage2; else ONLY=stage1; fi
rm -rf gpurun_out/r6s/$PART
TVQ_BENCH_ONLY=$ONLY timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6s/$PART -o p -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/r6s/$PART.log 2>&1 || { tail -20 gpurun_out/r6s/$PART.log; exit 1; }
T=$(find gpurun_out/r6s/$PART -name "*kernel_trace.csv" | head -1)
python tools/step_timeline.py "$T" 2 40 gpurun_out/r6s/seq_$PART.txt > gpurun_out/r6s/timeline_$PART.txt
python tools/step_table.py "$T" 5 gpurun_out/r6s/table_$PART.csv > gpurun_out/r6s/table_$PART.txt
head -12 gpurun_out/r6s/timeline_$PART.txt
rm -rf gpurun_out/r6s/$PART

#!/bin/bash
# Step kernel sequence per queue (rocprofv3 kernel trace of graph-replayed joint steps).
set -o pipefail
mkdir -p gpurun_out/seq
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/seq/step
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/seq/step -o step -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/seq/step.log 2>&1 || { tail -20 gpurun_out/seq/step.log; exit 1; }
T=$(find gpurun_out/seq/step -name "*kernel_trace.csv" | head -1)
python tools/step_timeline.py "$T" 2 8 gpurun_out/seq/seq.txt > gpurun_out/seq/timeline.txt
head -12 gpurun_out/seq/timeline.txt
grep '"value"' gpurun_out/seq/step.log | cut -c1-200

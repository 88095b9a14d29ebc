#!/bin/bash
# Evidence tables: the joint step's kernel table (rocprofv3 over graph-replayed steps) and
# the top kernel's roofline leg (LEG=rbbwd: kernel stats + FETCH/WRITE/SQ counter passes).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
rm -rf gpurun_out/prof_step3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_step3 -o step -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/prof_step3.log 2>&1 || { tail -20 gpurun_out/prof_step3.log; exit 1; }
T=$(find gpurun_out/prof_step3 -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/step_table.csv | head -5
python tools/step_timeline.py "$T" 2 12 > gpurun_out/step_timeline.txt
LEG=${LEG:-rbbwd} bash tools/gpu_roofline.sh

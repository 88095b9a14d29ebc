#!/bin/bash
# Round-4 evidence, part A (profiles of the tree named in tools/.tree): the joint step's
# kernel table (rocprofv3 over graph-replayed steps), the sampler batch's kernel table, and
# the PMC traffic of every roofline leg bench.py reports.  Copy into profiles/ afterwards.
set -o pipefail
mkdir -p gpurun_out/r4ev
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
rm -rf gpurun_out/r4ev/step
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ev/step -o step -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/r4ev/step.log 2>&1 || { tail -20 gpurun_out/r4ev/step.log; exit 1; }
T=$(find gpurun_out/r4ev/step -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r4ev/step_kernel_stats.csv > /dev/null
head -4 gpurun_out/r4ev/step_kernel_stats.csv
rm -rf gpurun_out/r4ev/samp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ev/samp -o samp -- python tools/sampler_graph_prof.py 5 > gpurun_out/r4ev/samp.log 2>&1 || { tail -20 gpurun_out/r4ev/samp.log; exit 1; }
T=$(find gpurun_out/r4ev/samp -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r4ev/sampler_batch_kernels.csv add_i64_kernel > /dev/null
head -4 gpurun_out/r4ev/sampler_batch_kernels.csv
for LEG in dominant wgrad rbbwd vqassign linfwd t32; do
  LEG=$LEG bash tools/gpu_roofline.sh > gpurun_out/r4ev/roof_$LEG.log 2>&1 || { tail -20 gpurun_out/r4ev/roof_$LEG.log; exit 1; }
  echo "$LEG $(grep -o '"traffic_bytes": [0-9]*' gpurun_out/roof_$LEG/traffic.json)"
done
echo evidence-a-done

#!/bin/bash
# Round-5 evidence (profiles of the current tree): the joint step's kernel table (rocprofv3
# over graph-replayed steps), the sampler batch's kernel table, and the PMC traffic of every
# roofline leg bench.py reports.  Copy into profiles/ afterwards (tools/collect_r5.sh).
set -o pipefail
mkdir -p gpurun_out/r5ev
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
git_tree=$(cat tools/.tree 2>/dev/null || echo unknown)
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs"
rm -rf gpurun_out/r5ev/step
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ev/step -o step -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/r5ev/step.log 2>&1 || { tail -20 gpurun_out/r5ev/step.log; exit 1; }
T=$(find gpurun_out/r5ev/step -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r5ev/step_kernel_stats.csv > gpurun_out/r5ev/step_table.txt
python tools/step_timeline.py "$T" 2 15 > gpurun_out/r5ev/step_timeline.txt
head -2 gpurun_out/r5ev/step_table.txt
rm -f "$T"
rm -rf gpurun_out/r5ev/samp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ev/samp -o samp -- python tools/sampler_graph_prof.py 5 > gpurun_out/r5ev/samp.log 2>&1 || { tail -20 gpurun_out/r5ev/samp.log; exit 1; }
T=$(find gpurun_out/r5ev/samp -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r5ev/sampler_batch_kernels.csv add_i64_kernel > /dev/null
head -4 gpurun_out/r5ev/sampler_batch_kernels.csv
rm -f "$T"
for LEG in dominant wgrad rbbwd vqassign linfwd t32 attn n16 rb64; do
  LEG=$LEG bash tools/gpu_roofline.sh > gpurun_out/r5ev/roof_$LEG.log 2>&1 || { tail -20 gpurun_out/r5ev/roof_$LEG.log; exit 1; }
  echo "$LEG $(grep -o '"traffic_bytes": [0-9]*' gpurun_out/roof_$LEG/traffic.json)"
done
echo evidence-done

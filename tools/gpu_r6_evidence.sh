#!/bin/bash
# Round-6 evidence (profiles of the current tree): the joint step's kernel table (rocprofv3
# over graph-replayed steps), the sampler batch's kernel table, and the PMC traffic of every
# roofline leg bench.py reports.  Copy into profiles/ afterwards (tools/collect_r6.sh).
set -o pipefail
mkdir -p gpurun_out/r6ev
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
git_tree=$(cat tools/.tree 2>/dev/null || echo unknown)
PART=${PART:-all}  # A: tests, smoke, bench, step / sampler tables; B: the roofline legs
if [ "$PART" != B ]; then
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r6ev/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r6ev/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r6ev/pytest_gpu.log
timeout -k 10 600 python __graft_entry__.py smoke > gpurun_out/r6ev/smoke.log 2>&1 || { tail -20 gpurun_out/r6ev/smoke.log; exit 1; }
tail -4 gpurun_out/r6ev/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r6ev/bench.log 2>&1 || { tail -20 gpurun_out/r6ev/bench.log; exit 1; }
tail -1 gpurun_out/r6ev/bench.log | cut -c1-300
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs"
rm -rf gpurun_out/r6ev/step
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6ev/step -o step -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/r6ev/step.log 2>&1 || { tail -20 gpurun_out/r6ev/step.log; exit 1; }
T=$(find gpurun_out/r6ev/step -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r6ev/step_kernel_stats.csv > gpurun_out/r6ev/step_table.txt
python tools/step_timeline.py "$T" 2 15 > gpurun_out/r6ev/step_timeline.txt
head -2 gpurun_out/r6ev/step_table.txt
rm -f "$T"
rm -rf gpurun_out/r6ev/samp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6ev/samp -o samp -- python tools/sampler_graph_prof.py 5 > gpurun_out/r6ev/samp.log 2>&1 || { tail -20 gpurun_out/r6ev/samp.log; exit 1; }
T=$(find gpurun_out/r6ev/samp -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r6ev/sampler_batch_kernels.csv add_i64_kernel > /dev/null
head -4 gpurun_out/r6ev/sampler_batch_kernels.csv
rm -f "$T"
fi
[ "$PART" = A ] && { echo evidence-A-done; exit 0; }
for LEG in dominant wgrad rbbwd rb32bwd vqassign linfwd t32 attn n16 rb64; do
  LEG=$LEG bash tools/gpu_roofline.sh > gpurun_out/r6ev/roof_$LEG.log 2>&1 || { tail -20 gpurun_out/r6ev/roof_$LEG.log; exit 1; }
  echo "$LEG $(grep -o '"traffic_bytes": [0-9]*' gpurun_out/roof_$LEG/traffic.json)"
done
echo evidence-done

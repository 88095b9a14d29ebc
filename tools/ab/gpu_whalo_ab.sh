#!/bin/bash
# conv_wgrad_halo slab cap A/B: the wgrad leg alone and the step.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for v in 4194304 1048576 2097152 8388608 16777216; do
  TVQ_WHALO_SLAB_MAX=$v timeout -k 10 120 python tools/roofline_only.py wgrad > gpurun_out/wh_$v.json 2>&1 || { tail -5 gpurun_out/wh_$v.json; exit 1; }
  TVQ_WHALO_SLAB_MAX=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/bench_wh.log 2>&1 || { tail -20 gpurun_out/bench_wh.log; exit 1; }
  echo "cap=$v leg $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/wh_$v.json) step $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_wh.log)"
done

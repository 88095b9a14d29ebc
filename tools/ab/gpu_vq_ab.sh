#!/bin/bash
# VQ assign row groups per workgroup: VQ tests, the VQ leg per TVQ_VQ_RG, the step alternated
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_vq.py tests/test_stage1.py tests/test_stage2_golden.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/vq_tests.log 2>&1 || { tail -30 gpurun_out/vq_tests.log; exit 1; }
tail -2 gpurun_out/vq_tests.log
for rg in 0 4 3 2; do
  TVQ_VQ_RG=$rg timeout -k 10 120 python tools/roofline_only.py vqassign > gpurun_out/vq_leg.log 2>&1 || { tail -5 gpurun_out/vq_leg.log; exit 1; }
  echo "rg=$rg $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/vq_leg.log)"
done
B="python bench.py --steps 50 --warmup 10 --no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2 3; do
  for rg in 0 4; do
    TVQ_VQ_RG=$rg timeout -k 10 300 $B > gpurun_out/ab_vq.log 2>&1 || { tail -20 gpurun_out/ab_vq.log; exit 1; }
    echo "rg=$rg $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_vq.log)"
  done
done

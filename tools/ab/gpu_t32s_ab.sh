#!/bin/bash
# 16-channel -> 128 convs on the 32x32-MFMA tile: conv tests, the shapes with TVQ_T32_SMALLC=1/0,
# then the step alternated (env switch)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TVQ_T32_SMALLC=1 timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py tests/test_stage1.py -x -q -m gpu -k "conv or stage1" \
  --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for v in 1 0; do
  echo "[TVQ_T32_SMALLC=$v]"
  TVQ_T32_SMALLC=$v timeout -k 10 200 python tools/conv_shapes_bench.py 6,7,13,14,17,18 > gpurun_out/t32s_shapes.log 2>&1 || { tail -5 gpurun_out/t32s_shapes.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/t32s_shapes.log
done
B="python bench.py --steps 50 --warmup 10 --no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2 3; do
  TVQ_T32_SMALLC=1 timeout -k 10 300 $B > gpurun_out/ab_new_$i.log 2>&1 || { tail -20 gpurun_out/ab_new_$i.log; exit 1; }
  echo "new $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_new_$i.log)"
  TVQ_T32_SMALLC=0 timeout -k 10 300 $B > gpurun_out/ab_old_$i.log 2>&1 || { tail -20 gpurun_out/ab_old_$i.log; exit 1; }
  echo "old $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_old_$i.log)"
done

#!/bin/bash
# Small-channel stride-2 conv weight gradient: conv / stage tests, the affected shapes new vs $OLD, then
# the step alternated new / $OLD
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OLD=${OLD:-t-vq-vae-trajgen_amd/lib_ab/libtvq_hip_cvold.so}
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py tests/test_stage1.py tests/test_stage2_golden.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/wt_tests.log 2>&1 || { tail -30 gpurun_out/wt_tests.log; exit 1; }
tail -2 gpurun_out/wt_tests.log
for cfg in "lib/libtvq_hip.so 256" "lib/libtvq_hip.so 512" "lib/libtvq_hip.so 1024" "lib_ab/libtvq_hip_cvold.so 0"; do
  set -- $cfg; lib=t-vq-vae-trajgen_amd/$1
  echo "[$cfg]"
  TVQ_WSMALL_S=$2 TVQ_HIP_LIB=$lib timeout -k 10 200 python tools/conv_shapes_bench.py 0,2,3,19,20,21,22 > gpurun_out/wt_shapes.log 2>&1 || { tail -5 gpurun_out/wt_shapes.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/wt_shapes.log
done
B="python bench.py --steps 50 --warmup 10 --no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/ab_new_$i.log 2>&1 || { tail -20 gpurun_out/ab_new_$i.log; exit 1; }
  echo "new $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_new_$i.log)"
  TVQ_HIP_LIB=$OLD timeout -k 10 300 $B > gpurun_out/ab_old_$i.log 2>&1 || { tail -20 gpurun_out/ab_old_$i.log; exit 1; }
  echo "old $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_old_$i.log)"
done

#!/bin/bash
# Stride-2 conv kernels walking segments: tests, shapes per block cap (TVQ_S2_WG) vs $OLD,
# then the step alternated new / $OLD
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OLD=${OLD:-t-vq-vae-trajgen_amd/lib_ab/libtvq_hip_head.so}
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py -x -q -m gpu -k "conv" \
  --timeout 120 --timeout-method thread > gpurun_out/s2_tests.log 2>&1 || { tail -30 gpurun_out/s2_tests.log; exit 1; }
tail -1 gpurun_out/s2_tests.log
for cfg in "lib/libtvq_hip.so 256" "lib/libtvq_hip.so 512" "lib/libtvq_hip.so 1024" "lib/libtvq_hip.so 0" "lib_ab/libtvq_hip_head.so 0"; do
  set -- $cfg
  echo "[$cfg]"
  TVQ_S2_WG=$2 TVQ_HIP_LIB=t-vq-vae-trajgen_amd/$1 timeout -k 10 200 python tools/conv_shapes_bench.py 0,2,3,19,20,21,22 > gpurun_out/s2_shapes.log 2>&1 || { tail -5 gpurun_out/s2_shapes.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/s2_shapes.log
done

#!/bin/bash
# conv_small channel pipelining (+ TVQ_CONV_SMALL_F=1 forward gathers): conv / stage tests,
# every step conv shape new / $OLD / new+small_f, then the step alternated
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OLD=${OLD:-t-vq-vae-trajgen_amd/lib_ab/libtvq_hip_cvold.so}
NEW=t-vq-vae-trajgen_amd/lib/libtvq_hip.so
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py tests/test_stage1.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/sm_tests.log 2>&1 || { tail -30 gpurun_out/sm_tests.log; exit 1; }
tail -2 gpurun_out/sm_tests.log
TVQ_CONV_SMALL_F=1 timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py -x -q -m gpu -k conv \
  --timeout 120 --timeout-method thread > gpurun_out/sm_tests_f.log 2>&1 || { tail -30 gpurun_out/sm_tests_f.log; exit 1; }
tail -2 gpurun_out/sm_tests_f.log
for c in "$NEW 0" "$OLD 0" "$NEW 1"; do
  set -- $c
  echo "[$1 small_f=$2]"
  TVQ_CONV_SMALL_F=$2 TVQ_HIP_LIB=$1 timeout -k 10 300 python tools/conv_shapes_bench.py > gpurun_out/sm_shapes.log 2>&1 || { tail -5 gpurun_out/sm_shapes.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/sm_shapes.log
done
B="python bench.py --steps 50 --warmup 10 --no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2; do
  for c in "$NEW 0" "$OLD 0" "$NEW 1"; do
    set -- $c
    TVQ_CONV_SMALL_F=$2 TVQ_HIP_LIB=$1 timeout -k 10 300 $B > gpurun_out/ab_sm.log 2>&1 || { tail -20 gpurun_out/ab_sm.log; exit 1; }
    echo "[$1 small_f=$2] $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_sm.log)"
  done
done

#!/bin/bash
# One change: its tests ($TESTS, -k $TK), then the step alternated new / $OLD (3 pairs)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OLD=${OLD:-t-vq-vae-trajgen_amd/lib_ab/libtvq_hip_head.so}
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_ops_gpu.py} -x -q -m gpu ${TK:+-k "$TK"} \
  --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
B="python bench.py --steps 50 --warmup 10 --no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/ab_new_$i.log 2>&1 || { tail -20 gpurun_out/ab_new_$i.log; exit 1; }
  echo "new $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_new_$i.log)"
  TVQ_HIP_LIB=$OLD timeout -k 10 300 $B > gpurun_out/ab_old_$i.log 2>&1 || { tail -20 gpurun_out/ab_old_$i.log; exit 1; }
  echo "old $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_old_$i.log)"
done

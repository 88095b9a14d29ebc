#!/bin/bash
# BN whole-channel kernels: BN / stage tests, then the step with TVQ_BN_CHAN=1 / 0 alternated
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py tests/test_stage1.py tests/test_stage2.py tests/test_stage2_golden.py tests/test_resblock.py tests/test_graph.py tests/test_dp_gpu.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/bn_tests.log 2>&1 || { tail -30 gpurun_out/bn_tests.log; exit 1; }
tail -2 gpurun_out/bn_tests.log
B="python bench.py --steps 50 --warmup 10 --no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2 3; do
  for v in 1 0; do
    TVQ_BN_CHAN=$v timeout -k 10 300 $B > gpurun_out/ab_bn$v.log 2>&1 || { tail -20 gpurun_out/ab_bn$v.log; exit 1; }
    echo "bn_chan=$v $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_bn$v.log)"
  done
done

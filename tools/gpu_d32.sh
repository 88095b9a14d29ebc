#!/bin/bash
# direct 3x3 conv: conv tests, step bench with / without it.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_resblock.py tests/test_stage1.py tests/test_graph.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/d32_tests.log 2>&1 || { tail -30 gpurun_out/d32_tests.log; exit 1; }
tail -2 gpurun_out/d32_tests.log
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for v in 1 0 1; do
  TVQ_CONV_D32=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/bench_d32_$v.log 2>&1 || { tail -20 gpurun_out/bench_d32_$v.log; exit 1; }
  echo "d32=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_d32_$v.log)"
done

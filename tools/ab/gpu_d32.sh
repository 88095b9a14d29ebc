#!/bin/bash
# direct conv: conv tests, step bench A/B over TVQ_CONV_D32 (max positions) / _NW.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_resblock.py tests/test_stage1.py tests/test_graph.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/d32_tests.log 2>&1 || { tail -30 gpurun_out/d32_tests.log; exit 1; }
tail -2 gpurun_out/d32_tests.log
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for v in ${D32_CASES:-"8192:4" "0:4" "8192:8" "32768:4"}; do
  TVQ_CONV_D32=${v%%:*} TVQ_CONV_D32_NW=${v##*:} timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/bench_d32.log 2>&1 || { tail -20 gpurun_out/bench_d32.log; exit 1; }
  echo "d32=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_d32.log)"
done

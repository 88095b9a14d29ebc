#!/bin/bash
# VQ / embedding / stage tests (segment sums, token rows), then a step-only bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_vq.py tests/test_stage1.py tests/test_stage2.py tests/test_stage2_golden.py tests/test_graph.py tests/test_dp_gpu.py tests/test_ops_gpu.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/vqseg_tests.log 2>&1 || { tail -30 gpurun_out/vqseg_tests.log; exit 1; }
tail -2 gpurun_out/vqseg_tests.log
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/bench_step.log 2>&1 || { tail -20 gpurun_out/bench_step.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_step.log

#!/bin/bash
# fused ResBlock tests + step bench + sampler leg
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_resblock.py tests/test_stage1.py tests/test_stage2.py tests/test_sampler.py tests/test_graph.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/rb_tests.log 2>&1 || { tail -30 gpurun_out/rb_tests.log; exit 1; }
tail -2 gpurun_out/rb_tests.log
STEPARGS="--no-roofline --no-config0 --no-cpu-baseline"
timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/bench_step.log 2>&1 || { tail -20 gpurun_out/bench_step.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"ms_per_batch": [0-9.]*' gpurun_out/bench_step.log

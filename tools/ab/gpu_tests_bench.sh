#!/bin/bash
# Every -m gpu test (one process), then a step-only bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-sampler --no-roofline --no-config0 --no-cpu-baseline > gpurun_out/bench_step.log 2>&1 || { tail -20 gpurun_out/bench_step.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_step.log

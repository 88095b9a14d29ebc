#!/bin/bash
# GEMM parity, step-only bench, then a step-only rocprofv3 kernel trace (timeline + table).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -m gpu -k "gemm or linear" \
  --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/bench_step.log 2>&1 || { tail -20 gpurun_out/bench_step.log; exit 1; }
tail -1 gpurun_out/bench_step.log | cut -c1-400
rm -rf gpurun_out/prof_step3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_step3 -o step -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/prof_step3.log 2>&1 || { tail -20 gpurun_out/prof_step3.log; exit 1; }
T=$(find gpurun_out/prof_step3 -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/step_table.csv | head -5
python tools/step_timeline.py "$T" 2 12 > gpurun_out/step_timeline.txt
head -60 gpurun_out/step_timeline.txt

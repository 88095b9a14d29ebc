#!/bin/bash
# Round 5 first run: every GPU test (flip counts printed), the step-only bench with the
# per-stage legs, a step kernel trace -> per-step table.
set -o pipefail
mkdir -p gpurun_out/r5a
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -q -m gpu -x -rP --timeout 120 --timeout-method thread > gpurun_out/r5a/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r5a/pytest_gpu.log; grep "flips=" gpurun_out/r5a/pytest_gpu.log > gpurun_out/r5a/flips.txt; [ $rc -eq 0 ] || exit $rc
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/r5a/bench_step.log 2>&1 || { tail -20 gpurun_out/r5a/bench_step.log; exit 1; }
tail -1 gpurun_out/r5a/bench_step.log | cut -c1-1500
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5a/prof -o step -- python bench.py --steps 5 --warmup 2 --no-stage-legs $STEPARGS > gpurun_out/r5a/prof.log 2>&1 || { tail -20 gpurun_out/r5a/prof.log; exit 1; }
T=$(find gpurun_out/r5a/prof -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r5a/step_table.csv | head -5
rm -f "$T"
echo r5a-done

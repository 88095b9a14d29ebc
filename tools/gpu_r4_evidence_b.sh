#!/bin/bash
# Round-4 evidence, part B: every -m gpu test, smoke(), then the full bench line (all legs,
# reading part A's profiles for the traffic / CU-weighted fields).
set -o pipefail
mkdir -p gpurun_out/r4ev
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r4ev/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r4ev/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4ev/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4ev/smoke.log 2>&1 || { tail -20 gpurun_out/r4ev/smoke.log; exit 1; }
tail -1 gpurun_out/r4ev/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r4ev/bench_full.log 2>&1 || { tail -20 gpurun_out/r4ev/bench_full.log; exit 1; }
tail -1 gpurun_out/r4ev/bench_full.log > gpurun_out/r4ev/bench_full.json
echo evidence-b-done

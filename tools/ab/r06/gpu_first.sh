#!/bin/bash
# Round-6 first GPU pass: every -m gpu test, the default bench line, and bench.py's own
# N = 2 launcher in rehearsal form (both ranks on cuda:0 over gloo).
set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/r6/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r6/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/r6/bench.log 2>&1 || { tail -20 gpurun_out/r6/bench.log; exit 1; }
tail -c 600 gpurun_out/r6/bench.log
TVQ_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs > gpurun_out/r6/bench2.log 2>&1 || { tail -20 gpurun_out/r6/bench2.log; exit 1; }
tail -c 400 gpurun_out/r6/bench2.log

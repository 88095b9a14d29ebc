#!/bin/bash
# GPU round check: every -m gpu test (one process, per-test timeout), then smoke, then a
# short bench.  Test failures (rc 1) do not stop the later steps; a crash, abort or time
# limit (any other rc) ends the call there.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 ${TVQ_TEST_TIMEOUT:-900} python -u -m pytest tests -v -m gpu --timeout 120 \
  --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ -n "$SKIP_SMOKE" ] || { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/smoke.log 2>&1; src=$?; tail -5 gpurun_out/smoke.log; [ $src -eq 0 ] || exit $src; }
[ -n "$SKIP_BENCH" ] || { timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-20} --warmup 5 \
  ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; brc=$?; tail -3 gpurun_out/bench.log; [ $brc -eq 0 ] || exit $brc; }
exit $rc

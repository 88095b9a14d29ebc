#!/bin/bash
# tests -> bench -> rocprof(kernel stats) ; each step time-limited; stop at first failure
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -40 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ -n "$CONTINUE_ON_TEST_FAIL" ] || exit $rc
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-20} --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof -name "*stats*" | head
exit $rc

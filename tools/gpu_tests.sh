#!/bin/bash
# GPU parity run: every -m gpu test, one process, bounded.
mkdir -p gpurun_out
timeout -k 10 ${TVQ_TEST_TIMEOUT:-900} python -m pytest tests -q -m gpu ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -60 gpurun_out/pytest_gpu.log
exit $rc

#!/bin/bash
# Round 4: the full-size parity tests, then a short bench (step only).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_fullsize_parity.py > gpurun_out/r4a_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4a_pytest.log
tail -30 gpurun_out/r4a_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-sampler --no-roofline --no-config0 --no-cpu-baseline > gpurun_out/r4a_bench.log 2>&1
rc2=$?
tail -3 gpurun_out/r4a_bench.log
exit $rc2

#!/bin/bash
# A/B: gpu tests (unless NOTEST), then bench variants given as env strings in $VARIANTS
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit $rc
fi
i=0
for v in ${VARIANTS:-"X=1"}; do
  i=$((i+1))
  env ${v//+/ } timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_$i.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/bench_$i.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["losses"])')"
  [ $rc -eq 0 ] || exit $rc
done

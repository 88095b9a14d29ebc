#!/bin/bash
# selected GPU tests ($TESTS) then one bench line with the sampler
set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > gpurun_out/r6/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6/quick_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r6/quick_tests.log | head -30; exit $rc; }
show() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['ms_per_step'],d.get('stage1_ms_per_step'),d.get('stage2_ms_per_step'),d['sampler']['ms_per_batch'])"; }
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-roofline --no-config0 --no-cpu-baseline > gpurun_out/r6/quick_bench.log 2>&1 || { tail -5 gpurun_out/r6/quick_bench.log; exit 1; }
echo "bench $(show gpurun_out/r6/quick_bench.log)"
done

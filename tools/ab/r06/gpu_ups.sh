#!/bin/bash
# Upscale token-grid conv: its tests + the stage2 / sampler suites, then A/B of the joint step,
# the per-stage legs and the sampler batch (TVQ_UPS_TOKENS=0: upsample -> conv).
set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_upscale.py tests/test_stage2.py tests/test_stage2_golden.py tests/test_sampler.py tests/test_sampler_full.py tests/test_fullsize_parity.py tests/test_prior_eval.py > gpurun_out/r6/ups_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6/ups_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r6/ups_tests.log | head -30; exit $rc; }
show() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['ms_per_step'],d.get('stage1_ms_per_step'),d.get('stage2_ms_per_step'),d['sampler']['ms_per_batch'])"; }
ARGS="--steps 40 --warmup 5 --no-roofline --no-config0 --no-cpu-baseline"
for rep in 1 2; do
  for v in 1 0; do
    TVQ_UPS_TOKENS=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/r6/ups_$v.log 2>&1 || { tail -5 gpurun_out/r6/ups_$v.log; exit 1; }
    echo "UPS_TOKENS=$v $(show gpurun_out/r6/ups_$v.log)"
  done
done

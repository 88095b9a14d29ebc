#!/bin/bash
# BN statistics in the stride-2 conv epilogue: tests, then A/B of the joint step (TVQ_BN_STATS).
set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bn_stats.py tests/test_stage1.py tests/test_fullsize_parity.py tests/test_graph.py tests/test_conv_bn_eval.py > gpurun_out/r6/bns_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6/bns_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r6/bns_tests.log | head -30; exit $rc; }
show() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['ms_per_step'],d.get('stage1_ms_per_step'),d.get('stage2_ms_per_step'))"; }
ARGS="--steps 40 --warmup 5 --no-roofline --no-config0 --no-cpu-baseline --no-sampler"
for rep in 1 2 3; do
  for v in 1 0; do
    TVQ_BN_STATS=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/r6/bns_$v.log 2>&1 || { tail -5 gpurun_out/r6/bns_$v.log; exit 1; }
    echo "BN_STATS=$v $(show gpurun_out/r6/bns_$v.log)"
  done
done

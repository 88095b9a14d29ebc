#!/bin/bash
# ResBlock pair chain: its tests, then the A/B of TVQ_RESBLOCK_PAIR with the per-stage legs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resblock.py tests/test_fullsize_parity.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pair_tests.log 2>&1 || { tail -30 gpurun_out/pair_tests.log; exit 1; }
tail -3 gpurun_out/pair_tests.log
R5AB="TVQ_RESBLOCK_PAIR=0" bash tools/ab/r05/gpu_ab_stage.sh

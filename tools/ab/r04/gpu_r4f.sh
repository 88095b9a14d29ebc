#!/bin/bash
# Round 4: DP overlap form (BranchStepGraph) + per-id pack caches: the whole GPU suite and smoke.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --durations=25 \
  --timeout 240 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1 || { tail -60 gpurun_out/r4f_tests.log; exit 1; }
tail -30 gpurun_out/r4f_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4f_smoke.log 2>&1 || { tail -20 gpurun_out/r4f_smoke.log; exit 1; }
tail -1 gpurun_out/r4f_smoke.log

#!/bin/bash
# GPU tests only: R5TESTS (default: all of tests/), log under gpurun_out/${R5TAG}.
set -o pipefail
D=gpurun_out/${R5TAG:-r5t}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest ${R5TESTS:-tests} -q -m gpu -x --timeout 120 --timeout-method thread > $D/t.log 2>&1
rc=$?; tail -3 $D/t.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $D/t.log | tail -60; exit $rc; }

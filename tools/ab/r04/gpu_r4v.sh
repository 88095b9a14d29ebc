#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv_halo_cc.py > gpurun_out/r4v_tests.log 2>&1 || { tail -40 gpurun_out/r4v_tests.log; exit 1; }
tail -1 gpurun_out/r4v_tests.log
timeout -k 10 300 python tools/ab/r04/hcc_bench.py

#!/bin/bash
# DP branch replay order: the 2-process GPU DP tests, and the opt-in halo_cc tests
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_dp_gpu.py tests/test_conv_halo_cc.py tests/test_graph.py > gpurun_out/r4u_tests.log 2>&1 || { tail -40 gpurun_out/r4u_tests.log; exit 1; }
tail -1 gpurun_out/r4u_tests.log

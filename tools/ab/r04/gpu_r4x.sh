#!/bin/bash
# graphed sampler: LF decoder on a side stream during the HF pass (TVQ_SAMPLER_OVERLAP)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_sampler_full.py tests/test_sampler.py > gpurun_out/r4x_tests.log 2>&1 || { tail -40 gpurun_out/r4x_tests.log; exit 1; }
tail -1 gpurun_out/r4x_tests.log
for i in 1 2 3; do
for O in 1 0; do
TVQ_SAMPLER_OVERLAP=$O timeout -k 10 200 python tools/sampler_graph_prof.py 20 > gpurun_out/r4x_samp.log 2>&1 || { tail -20 gpurun_out/r4x_samp.log; exit 1; }
echo "overlap=$O $(tail -1 gpurun_out/r4x_samp.log)"
done
done

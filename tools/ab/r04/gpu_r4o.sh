#!/bin/bash
# prior/sampler GPU tests, then the sampler batch kernel table on the current tree
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_prior_eval.py tests/test_sampler.py tests/test_sampler_full.py > gpurun_out/r4o_tests.log 2>&1 || { tail -30 gpurun_out/r4o_tests.log; exit 1; }
tail -2 gpurun_out/r4o_tests.log
timeout -k 10 200 python tools/sampler_graph_prof.py 20 > gpurun_out/r4o_wall.log 2>&1 || { tail -20 gpurun_out/r4o_wall.log; exit 1; }
tail -3 gpurun_out/r4o_wall.log
rm -rf gpurun_out/r4o_samp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4o_samp -o samp -- python tools/sampler_graph_prof.py 5 > gpurun_out/r4o_samp.log 2>&1 || { tail -20 gpurun_out/r4o_samp.log; exit 1; }
T=$(find gpurun_out/r4o_samp -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r4o_sampler_batch.csv add_i64_kernel | head -16

#!/bin/bash
# fused eval conv + BN (+ Snake): tests, conv/sampler regressions, sampler batch table
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_bn_eval.py tests/test_sampler_full.py tests/test_ops_gpu.py tests/test_sampler.py > gpurun_out/r4p_tests.log 2>&1 || { tail -40 gpurun_out/r4p_tests.log; exit 1; }
tail -2 gpurun_out/r4p_tests.log
timeout -k 10 200 python tools/sampler_graph_prof.py 20 > gpurun_out/r4p_wall.log 2>&1 || { tail -20 gpurun_out/r4p_wall.log; exit 1; }
tail -1 gpurun_out/r4p_wall.log
TVQ_FUSED_BN_EVAL=0 timeout -k 10 200 python tools/sampler_graph_prof.py 20 > gpurun_out/r4p_wall0.log 2>&1 || { tail -20 gpurun_out/r4p_wall0.log; exit 1; }
tail -1 gpurun_out/r4p_wall0.log
rm -rf gpurun_out/r4p_samp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4p_samp -o samp -- python tools/sampler_graph_prof.py 5 > gpurun_out/r4p_samp.log 2>&1 || { tail -20 gpurun_out/r4p_samp.log; exit 1; }
T=$(find gpurun_out/r4p_samp -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r4p_sampler_batch.csv add_i64_kernel > gpurun_out/r4p_table.txt
head -30 gpurun_out/r4p_table.txt

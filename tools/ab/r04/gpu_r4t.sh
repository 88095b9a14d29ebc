#!/bin/bash
# channel-chunked halo conv (128 -> 16): tests, step A/B (TVQ_CONV_HCC), sampler A/B, table
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_conv_halo_cc.py tests/test_ops_gpu.py tests/test_stage1.py tests/test_fullsize_parity.py tests/test_conv_bn_eval.py tests/test_sampler_full.py > gpurun_out/r4t_tests.log 2>&1 || { tail -40 gpurun_out/r4t_tests.log; exit 1; }
tail -1 gpurun_out/r4t_tests.log
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2; do
for H in 1 0; do
TVQ_CONV_HCC=$H timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/r4t_bench.log 2>&1 || { tail -20 gpurun_out/r4t_bench.log; exit 1; }
echo "hcc=$H $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4t_bench.log)"
TVQ_CONV_HCC=$H timeout -k 10 200 python tools/sampler_graph_prof.py 20 > gpurun_out/r4t_samp.log 2>&1 || { tail -20 gpurun_out/r4t_samp.log; exit 1; }
echo "hcc=$H $(tail -1 gpurun_out/r4t_samp.log)"
done
done
rm -rf gpurun_out/r4t_step
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4t_step -o step -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/r4t_step.log 2>&1 || { tail -20 gpurun_out/r4t_step.log; exit 1; }
T=$(find gpurun_out/r4t_step -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r4t_step_table.csv > gpurun_out/r4t_table.txt
head -1 gpurun_out/r4t_table.txt
grep -E "halo_cc|16, 256" gpurun_out/r4t_step_table.csv

#!/bin/bash
# register-resident group-by scan: group-by / VQ / stage tests, step x3, step table rows
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_groupby.py tests/test_vq.py tests/test_stage1.py tests/test_stage2_golden.py tests/test_fullsize_parity.py tests/test_graph.py > gpurun_out/r4y_tests.log 2>&1 || { tail -40 gpurun_out/r4y_tests.log; exit 1; }
tail -1 gpurun_out/r4y_tests.log
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/r4y_bench.log 2>&1 || { tail -20 gpurun_out/r4y_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4y_bench.log
done
rm -rf gpurun_out/r4y_step
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4y_step -o step -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/r4y_step.log 2>&1 || { tail -20 gpurun_out/r4y_step.log; exit 1; }
T=$(find gpurun_out/r4y_step -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r4y_step_table.csv > gpurun_out/r4y_table.txt
head -1 gpurun_out/r4y_table.txt
grep -E "gb_" gpurun_out/r4y_step_table.csv

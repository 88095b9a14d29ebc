#!/bin/bash
# per-stream deferred reduction batches: graph / stage / dp tests, joint step x3, step table
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_graph.py tests/test_stage2.py tests/test_stage2_golden.py tests/test_stage1.py tests/test_dp_gpu.py tests/test_fused_ff.py > gpurun_out/r4s_tests.log 2>&1 || { tail -40 gpurun_out/r4s_tests.log; exit 1; }
tail -1 gpurun_out/r4s_tests.log
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/r4s_bench.log 2>&1 || { tail -20 gpurun_out/r4s_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4s_bench.log
done
rm -rf gpurun_out/r4s_step
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4s_step -o step -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/r4s_step.log 2>&1 || { tail -20 gpurun_out/r4s_step.log; exit 1; }
T=$(find gpurun_out/r4s_step -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r4s_step_table.csv > gpurun_out/r4s_table.txt
head -1 gpurun_out/r4s_table.txt
grep -E "reduce_rows" gpurun_out/r4s_step_table.csv

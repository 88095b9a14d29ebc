#!/bin/bash
# Round 4: fused tied-logits CE + group-by descriptors.  Tests, the step alternated
# fused CE / TVQ_FUSED_CE=0 x3, and the step kernel table.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_tied_ce.py tests/test_groupby.py tests/test_stage2_golden.py tests/test_stage2.py tests/test_fullsize_parity.py tests/test_vq.py tests/test_dp_gpu.py -x -q -m gpu \
  --timeout 240 --timeout-method thread > gpurun_out/r4e_tests.log 2>&1 || { tail -40 gpurun_out/r4e_tests.log; exit 1; }
tail -2 gpurun_out/r4e_tests.log
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
B="python bench.py --steps 100 --warmup 10 $STEPARGS"
for i in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/r4e_ab_new_$i.log 2>&1 || { tail -20 gpurun_out/r4e_ab_new_$i.log; exit 1; }
  echo "new $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4e_ab_new_$i.log)"
  TVQ_FUSED_CE=0 timeout -k 10 300 $B > gpurun_out/r4e_ab_old_$i.log 2>&1 || { tail -20 gpurun_out/r4e_ab_old_$i.log; exit 1; }
  echo "unfusedCE $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4e_ab_old_$i.log)"
done
rm -rf gpurun_out/r4e_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4e_prof -o step -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/r4e_prof.log 2>&1 || { tail -20 gpurun_out/r4e_prof.log; exit 1; }
T=$(find gpurun_out/r4e_prof -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r4e_step_table.csv > /dev/null
grep -E "ce_|seg_|gb_|masked|skinny" gpurun_out/r4e_step_table.csv

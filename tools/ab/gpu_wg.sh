#!/bin/bash
# Grouped weight-gradient GEMM: parity tests, the dominant leg at a few block targets,
# the graph/stage2/DP tests that run it inside a step, then a step-only bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -m gpu -k "wgrad or gemm" \
  --timeout 120 --timeout-method thread > gpurun_out/wg_tests.log 2>&1 || { tail -30 gpurun_out/wg_tests.log; exit 1; }
tail -2 gpurun_out/wg_tests.log
for b in ${WG_KSPAN:-256 512 1024}; do
  TVQ_WG_KSPAN=$b timeout -k 10 120 python tools/roofline_only.py dominant > gpurun_out/wg_dom_$b.json 2>&1 || { tail -20 gpurun_out/wg_dom_$b.json; exit 1; }
  echo "kspan $b: $(cut -c1-400 gpurun_out/wg_dom_$b.json | grep -o '"achieved[^,]*,\|"avg_launch_us[^,]*' | tr '\n' ' ')"
done
timeout -k 10 400 python -u -m pytest tests/test_graph.py tests/test_stage2.py tests/test_stage2_golden.py tests/test_stage1.py tests/test_dp_gpu.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/wg_step_tests.log 2>&1 || { tail -30 gpurun_out/wg_step_tests.log; exit 1; }
tail -2 gpurun_out/wg_step_tests.log
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for v in 1 0; do
  TVQ_WGRAD_GROUP=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/bench_step_wg$v.log 2>&1 || { tail -20 gpurun_out/bench_step_wg$v.log; exit 1; }
  echo "group=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_step_wg$v.log)"
done

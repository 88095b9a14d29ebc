#!/bin/bash
# Round 4: project_in folded into the LF prior's tables: sampling tests, sampler batch, and the
# joint step (3 runs) on the current tree.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_prior_eval.py tests/test_sampler.py tests/test_sampler_full.py -x -q -m gpu \
  --timeout 200 --timeout-method thread > gpurun_out/r4k_t1.log 2>&1 || { tail -60 gpurun_out/r4k_t1.log; exit 1; }
tail -2 gpurun_out/r4k_t1.log
for i in 1 2; do
  timeout -k 10 300 python tools/sampler_graph_prof.py 20 > gpurun_out/r4k_samp_$i.log 2>&1 || { tail -20 gpurun_out/r4k_samp_$i.log; exit 1; }
  echo "sampler $(tail -1 gpurun_out/r4k_samp_$i.log)"
done
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 $STEPARGS > gpurun_out/r4k_step_$i.log 2>&1 || { tail -20 gpurun_out/r4k_step_$i.log; exit 1; }
  echo "step $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4k_step_$i.log)"
done

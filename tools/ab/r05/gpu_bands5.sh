#!/bin/bash
# Round-5 attribution without a profiler: joint, each stage alone, each stage1 band alone,
# joint with one stage1 band (graph-replayed, 50 steps each).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 50 --warmup 10 --no-sampler --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs"
run() { # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 $B > gpurun_out/att_$n.log 2>&1 || { tail -20 gpurun_out/att_$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/att_$n.log)"
}
run joint TVQ_X=1
run stage1 TVQ_BENCH_ONLY=stage1
run stage2 TVQ_BENCH_ONLY=stage2
run stage1_LF TVQ_BENCH_ONLY=stage1 TVQ_BENCH_BANDS=LF
run stage1_HF TVQ_BENCH_ONLY=stage1 TVQ_BENCH_BANDS=HF
run joint_LFonly TVQ_BENCH_BANDS=LF
run joint_HFonly TVQ_BENCH_BANDS=HF
run joint2 TVQ_X=2

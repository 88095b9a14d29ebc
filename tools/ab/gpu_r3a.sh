#!/bin/bash
# Round 3: every -m gpu test, then the step A/B (acq_rel ticket vs relaxed ticket), then
# the stage1-only / stage2-only attribution (TVQ_BENCH_ONLY) -- step timings without a profiler.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 50 --warmup 10 --no-sampler --no-roofline --no-config0 --no-cpu-baseline"
REL=t-vq-vae-trajgen_amd/lib_ab/libtvq_hip_relaxed.so
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/ab_strict_$i.log 2>&1 || { tail -20 gpurun_out/ab_strict_$i.log; exit 1; }
  echo "strict $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_strict_$i.log)"
  TVQ_HIP_LIB=$REL timeout -k 10 300 $B > gpurun_out/ab_relaxed_$i.log 2>&1 || { tail -20 gpurun_out/ab_relaxed_$i.log; exit 1; }
  echo "relaxed $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_relaxed_$i.log)"
done
for o in stage1 stage2; do
  TVQ_BENCH_ONLY=$o timeout -k 10 300 $B > gpurun_out/only_$o.log 2>&1 || { tail -20 gpurun_out/only_$o.log; exit 1; }
  echo "only $o $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/only_$o.log)"
done

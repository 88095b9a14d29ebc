#!/bin/bash
# Round 4: fused feed-forward branch of the LF prior: its tests + the stage2 parity tests,
# then the joint step alternated fused / TVQ_FUSED_FF=0 (3 pairs) and stage2 alone.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_fused_ff.py tests/test_stage2.py tests/test_stage2_golden.py tests/test_fullsize_parity.py tests/test_graph.py tests/test_dp_gpu.py -x -q -m gpu \
  --timeout 200 --timeout-method thread > gpurun_out/r4m_t1.log 2>&1 || { tail -60 gpurun_out/r4m_t1.log; exit 1; }
tail -2 gpurun_out/r4m_t1.log
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 $STEPARGS > gpurun_out/r4m_new_$i.log 2>&1 || { tail -20 gpurun_out/r4m_new_$i.log; exit 1; }
  echo "fused $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4m_new_$i.log)"
  TVQ_FUSED_FF=0 timeout -k 10 300 python bench.py --steps 100 --warmup 10 $STEPARGS > gpurun_out/r4m_old_$i.log 2>&1 || { tail -20 gpurun_out/r4m_old_$i.log; exit 1; }
  echo "per-op $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4m_old_$i.log)"
done
for V in 1 0; do
  TVQ_FUSED_FF=$V TVQ_BENCH_ONLY=stage2 timeout -k 10 300 python bench.py --steps 100 --warmup 10 $STEPARGS > gpurun_out/r4m_s2_$V.log 2>&1 || { tail -20 gpurun_out/r4m_s2_$V.log; exit 1; }
  echo "stage2 alone fused=$V $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4m_s2_$V.log)"
done

#!/bin/bash
# GEMM epilogue-prefetch change: GEMM / stage2 tests, the Linear-forward leg new vs $OLD,
# then the step alternated new / $OLD
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OLD=${OLD:-t-vq-vae-trajgen_amd/lib_ab/libtvq_hip_gsold.so}
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_stage2.py tests/test_stage2_golden.py tests/test_prior_eval.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/ge_tests.log 2>&1 || { tail -30 gpurun_out/ge_tests.log; exit 1; }
tail -2 gpurun_out/ge_tests.log
for lib in t-vq-vae-trajgen_amd/lib/libtvq_hip.so $OLD; do
  TVQ_HIP_LIB=$lib timeout -k 10 120 python tools/roofline_only.py linfwd > gpurun_out/ge_leg.log 2>&1 || { tail -5 gpurun_out/ge_leg.log; exit 1; }
  echo "leg [$lib] $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/ge_leg.log)"
  TVQ_HIP_LIB=$lib timeout -k 10 200 python tools/gemm_bench.py lf_proj_train lf_logits_sampler lf_proj_sampler hf_proj_out_sampler > gpurun_out/ge_gb.log 2>&1 || { tail -5 gpurun_out/ge_gb.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/ge_gb.log | cut -c1-150
done
B="python bench.py --steps 50 --warmup 10 --no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/ab_new_$i.log 2>&1 || { tail -20 gpurun_out/ab_new_$i.log; exit 1; }
  echo "new $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_new_$i.log)"
  TVQ_HIP_LIB=$OLD timeout -k 10 300 $B > gpurun_out/ab_old_$i.log 2>&1 || { tail -20 gpurun_out/ab_old_$i.log; exit 1; }
  echo "old $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_old_$i.log)"
done
timeout -k 10 300 python tools/conv_shapes_bench.py > gpurun_out/conv_shapes.txt 2>&1 || { tail -5 gpurun_out/conv_shapes.txt; exit 1; }
cat gpurun_out/conv_shapes.txt | grep -v amdgpu.ids

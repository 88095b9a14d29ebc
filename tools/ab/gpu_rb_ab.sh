#!/bin/bash
# Fused ResBlock change: its tests, per-block phase timing (timing build), the ResBlock
# micro-bench on the new and the $OLD library, then the joint step alternated new / $OLD.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OLD=${OLD:-t-vq-vae-trajgen_amd/lib_ab/libtvq_hip_rbold.so}
export TVQ_HIP_LIB=${NEW:-t-vq-vae-trajgen_amd/lib/libtvq_hip.so}
NEWLIB=$TVQ_HIP_LIB
timeout -k 10 400 python -u -m pytest tests/test_resblock.py tests/test_stage1.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/rb_tests.log 2>&1 || { tail -30 gpurun_out/rb_tests.log; exit 1; }
tail -2 gpurun_out/rb_tests.log
timeout -k 10 120 python tools/rb_timing.py > gpurun_out/rb_timing.txt 2>&1 || { tail -20 gpurun_out/rb_timing.txt; exit 1; }
timeout -k 10 200 python tools/resblock_bench.py > gpurun_out/rb_bench_new.txt 2>&1 || { tail -20 gpurun_out/rb_bench_new.txt; exit 1; }
TVQ_HIP_LIB=$OLD timeout -k 10 200 python tools/resblock_bench.py > gpurun_out/rb_bench_old.txt 2>&1 || { tail -20 gpurun_out/rb_bench_old.txt; exit 1; }
echo new; cat gpurun_out/rb_bench_new.txt; echo old; cat gpurun_out/rb_bench_old.txt
B="python bench.py --steps 50 --warmup 10 --no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2 3; do
  TVQ_HIP_LIB=$NEWLIB timeout -k 10 300 $B > gpurun_out/ab_new_$i.log 2>&1 || { tail -20 gpurun_out/ab_new_$i.log; exit 1; }
  echo "new $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_new_$i.log)"
  TVQ_HIP_LIB=$OLD timeout -k 10 300 $B > gpurun_out/ab_old_$i.log 2>&1 || { tail -20 gpurun_out/ab_old_$i.log; exit 1; }
  echo "old $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_old_$i.log)"
done
O=gpurun_out/rbprof; mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o rb -- python tools/resblock_bench.py > $O/new.log 2>&1 || exit 1
TVQ_HIP_LIB=$OLD timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/old -o rb -- python tools/resblock_bench.py > $O/old.log 2>&1 || exit 1
echo prof-done

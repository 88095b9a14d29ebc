#!/bin/bash
# Round 4: ResBlock LDS bank layout.  Tests, ResBlock micro-bench new/old, the rbbwd roofline
# leg new/old with an SQ counter pass each, then the joint step alternated new/old x3.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OLD=t-vq-vae-trajgen_amd/lib_ab/libtvq_hip_rbold.so
timeout -k 10 500 python -u -m pytest tests/test_resblock.py tests/test_stage1.py tests/test_fullsize_parity.py -x -q -m gpu \
  --timeout 200 --timeout-method thread > gpurun_out/r4b_tests.log 2>&1 || { tail -30 gpurun_out/r4b_tests.log; exit 1; }
tail -2 gpurun_out/r4b_tests.log
timeout -k 10 200 python tools/resblock_bench.py > gpurun_out/r4b_rb_new.txt 2>&1 || { tail -20 gpurun_out/r4b_rb_new.txt; exit 1; }
TVQ_HIP_LIB=$OLD timeout -k 10 200 python tools/resblock_bench.py > gpurun_out/r4b_rb_old.txt 2>&1 || { tail -20 gpurun_out/r4b_rb_old.txt; exit 1; }
echo new; cat gpurun_out/r4b_rb_new.txt; echo old; cat gpurun_out/r4b_rb_old.txt
for v in new old; do
  L=t-vq-vae-trajgen_amd/lib/libtvq_hip.so; [ $v = old ] && L=$OLD
  TVQ_HIP_LIB=$L timeout -k 10 120 python tools/roofline_only.py rbbwd > gpurun_out/r4b_leg_$v.json 2>&1 || exit 1
  echo "$v $(cat gpurun_out/r4b_leg_$v.json | grep -o '"avg_launch_us": [0-9.]*')"
  TVQ_HIP_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/r4b_sq_$v -o roof -- python tools/roofline_only.py rbbwd > gpurun_out/r4b_sq_$v.log 2>&1 || exit 1
done
B="python bench.py --steps 50 --warmup 10 --no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/r4b_ab_new_$i.log 2>&1 || { tail -20 gpurun_out/r4b_ab_new_$i.log; exit 1; }
  echo "new $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4b_ab_new_$i.log)"
  TVQ_HIP_LIB=$OLD timeout -k 10 300 $B > gpurun_out/r4b_ab_old_$i.log 2>&1 || { tail -20 gpurun_out/r4b_ab_old_$i.log; exit 1; }
  echo "old $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4b_ab_old_$i.log)"
done

#!/bin/bash
# Round 4: ResBlock LDS bank layout + one-block group-by / one-launch segmented sums.
# Tests; ResBlock micro-bench and rbbwd leg (+SQ pass) new vs old ResBlock; the joint step
# alternated new / old-ResBlock / old-group-by x3.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RBOLD=t-vq-vae-trajgen_amd/lib_ab/libtvq_hip_rbold.so
GBOLD=t-vq-vae-trajgen_amd/lib_ab/libtvq_hip_gbold.so
NEW=t-vq-vae-trajgen_amd/lib/libtvq_hip.so
timeout -k 10 600 python -u -m pytest tests/test_groupby.py tests/test_prior_eval.py tests/test_sampler_full.py tests/test_resblock.py tests/test_stage1.py tests/test_fullsize_parity.py tests/test_vq.py tests/test_stage2.py tests/test_stage2_golden.py -x -q -m gpu \
  --timeout 200 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1 || { tail -30 gpurun_out/r4c_tests.log; exit 1; }
tail -2 gpurun_out/r4c_tests.log
timeout -k 10 200 python tools/resblock_bench.py > gpurun_out/r4c_rb_new.txt 2>&1 || { tail -20 gpurun_out/r4c_rb_new.txt; exit 1; }
TVQ_HIP_LIB=$RBOLD timeout -k 10 200 python tools/resblock_bench.py > gpurun_out/r4c_rb_old.txt 2>&1 || { tail -20 gpurun_out/r4c_rb_old.txt; exit 1; }
echo new; cat gpurun_out/r4c_rb_new.txt; echo old; cat gpurun_out/r4c_rb_old.txt
for v in new old; do
  L=$NEW; [ $v = old ] && L=$RBOLD
  TVQ_HIP_LIB=$L timeout -k 10 120 python tools/roofline_only.py rbbwd > gpurun_out/r4c_leg_$v.json 2>&1 || exit 1
  echo "$v $(cat gpurun_out/r4c_leg_$v.json | grep -o '"avg_launch_us": [0-9.]*')"
  TVQ_HIP_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/r4c_sq_$v -o roof -- python tools/roofline_only.py rbbwd > gpurun_out/r4c_sq_$v.log 2>&1 || exit 1
done
timeout -k 10 200 python tools/aten_sources.py > gpurun_out/r4c_aten_step.txt 2>&1 || { tail -20 gpurun_out/r4c_aten_step.txt; exit 1; }
timeout -k 10 200 python tools/aten_sources.py sampler > gpurun_out/r4c_aten_sampler.txt 2>&1 || { tail -20 gpurun_out/r4c_aten_sampler.txt; exit 1; }
echo aten-step; cat gpurun_out/r4c_aten_step.txt; echo aten-sampler; cat gpurun_out/r4c_aten_sampler.txt
B="python bench.py --steps 50 --warmup 10 --no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for i in 1 2 3; do
  for v in new rbold gbold; do
    L=$NEW; [ $v = rbold ] && L=$RBOLD; [ $v = gbold ] && L=$GBOLD
    TVQ_HIP_LIB=$L timeout -k 10 300 $B > gpurun_out/r4c_ab_${v}_$i.log 2>&1 || { tail -20 gpurun_out/r4c_ab_${v}_$i.log; exit 1; }
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4c_ab_${v}_$i.log)"
  done
done

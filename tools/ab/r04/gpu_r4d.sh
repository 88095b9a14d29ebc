#!/bin/bash
# Round 4 checkpoint: every GPU test, smoke, the step kernel table (rocprofv3), and the
# joint step alternated new / old group-by x3.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GBOLD=t-vq-vae-trajgen_amd/lib_ab/libtvq_hip_gbold.so
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r4d_tests.log 2>&1 || { tail -30 gpurun_out/r4d_tests.log; exit 1; }
tail -2 gpurun_out/r4d_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4d_smoke.log 2>&1 || { tail -20 gpurun_out/r4d_smoke.log; exit 1; }
tail -3 gpurun_out/r4d_smoke.log
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
rm -rf gpurun_out/r4d_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4d_prof -o step -- python bench.py --steps 5 --warmup 2 $STEPARGS > gpurun_out/r4d_prof.log 2>&1 || { tail -20 gpurun_out/r4d_prof.log; exit 1; }
T=$(find gpurun_out/r4d_prof -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r4d_step_table.csv > /dev/null
head -40 gpurun_out/r4d_step_table.csv
B="python bench.py --steps 100 --warmup 10 $STEPARGS"
for i in 1 2 3; do
  for v in new gbold; do
    L=t-vq-vae-trajgen_amd/lib/libtvq_hip.so; [ $v = gbold ] && L=$GBOLD
    TVQ_HIP_LIB=$L timeout -k 10 300 $B > gpurun_out/r4d_ab_${v}_$i.log 2>&1 || { tail -20 gpurun_out/r4d_ab_${v}_$i.log; exit 1; }
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4d_ab_${v}_$i.log)"
  done
done

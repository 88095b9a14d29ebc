#!/bin/bash
# RB<32,16> external weight gradients: tests, then the joint step vs the previous library
# (lib_ab/libtvq_hip_base.so), then the HW-queue count A/B.
set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resblock.py tests/test_fullsize_parity.py tests/test_stage1.py tests/test_graph.py > gpurun_out/r6/wext_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6/wext_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r6/wext_tests.log | head -30; exit $rc; }
show() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['ms_per_step'],d.get('stage1_ms_per_step'),d.get('stage2_ms_per_step'))"; }
ARGS="--steps 40 --warmup 5 --no-roofline --no-config0 --no-cpu-baseline --no-sampler"
for rep in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then E="TVQ_HIP_LIB=$GRAFT_REPO_ROOT/t-vq-vae-trajgen_amd/lib_ab/libtvq_hip_base.so"; else E="X=1"; fi
    env $E timeout -k 10 300 python bench.py $ARGS > gpurun_out/r6/wext_$v.log 2>&1 || { tail -5 gpurun_out/r6/wext_$v.log; exit 1; }
    echo "$v $(show gpurun_out/r6/wext_$v.log)"
  done
done
for q in 8 16 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py $ARGS > gpurun_out/r6/hwq_$q.log 2>&1 || { tail -5 gpurun_out/r6/hwq_$q.log; exit 1; }
  echo "HWQ=$q $(show gpurun_out/r6/hwq_$q.log)"
done

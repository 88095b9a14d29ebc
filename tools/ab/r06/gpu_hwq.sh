#!/bin/bash
# A/B of the number of HIP hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4):
# joint step, per-stage legs.
set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
show() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['ms_per_step'],d.get('stage1_ms_per_step'),d.get('stage2_ms_per_step'))"; }
ARGS="--steps 40 --warmup 5 --no-roofline --no-config0 --no-cpu-baseline --no-sampler"
for rep in 1 2; do
  for q in ${QS:-4 8 16}; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py $ARGS > gpurun_out/r6/hwq_$q.log 2>&1 || { tail -5 gpurun_out/r6/hwq_$q.log; exit 1; }
    echo "HWQ=$q $(show gpurun_out/r6/hwq_$q.log)"
  done
done

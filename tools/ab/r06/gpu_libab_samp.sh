#!/bin/bash
# sampler A/B of two library builds on one box: in-tree (base) vs lib_ab (variant), alternated
# processes (bench sampler leg only)
set -o pipefail
mkdir -p gpurun_out/libab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
show() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['sampler']['ms_per_batch'])"; }
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs > gpurun_out/libab/base.log 2>&1 || { tail -5 gpurun_out/libab/base.log; exit 1; }
  echo "base $(show gpurun_out/libab/base.log)"
  TVQ_HIP_LIB=$GRAFT_REPO_ROOT/lib_ab/libtvq_hip.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs > gpurun_out/libab/new.log 2>&1 || { tail -5 gpurun_out/libab/new.log; exit 1; }
  echo "new  $(show gpurun_out/libab/new.log)"
done

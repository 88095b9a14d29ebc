#!/bin/bash
# A/B of two library builds on one box: lib_ab/libtvq_hip.so (base) against the in-tree build,
# alternated (bench step legs + sampler), each run in its own process
set -o pipefail
mkdir -p gpurun_out/libab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
show() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['ms_per_step'],d.get('stage1_ms_per_step'),d.get('stage2_ms_per_step'),d['sampler']['ms_per_batch'])"; }
for rep in 1 2; do
  TVQ_HIP_LIB=$GRAFT_REPO_ROOT/lib_ab/libtvq_hip.so timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-roofline --no-config0 --no-cpu-baseline > gpurun_out/libab/base.log 2>&1 || { tail -5 gpurun_out/libab/base.log; exit 1; }
  echo "base $(show gpurun_out/libab/base.log)"
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-roofline --no-config0 --no-cpu-baseline > gpurun_out/libab/new.log 2>&1 || { tail -5 gpurun_out/libab/new.log; exit 1; }
  echo "new  $(show gpurun_out/libab/new.log)"
done

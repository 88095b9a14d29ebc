#!/bin/bash
# A/B of a runtime environment variable ($ABENV, e.g. HIP_FORCE_DEV_KERNARG=1) on the bench
# step and sampler legs, alternated processes on one box
set -o pipefail
mkdir -p gpurun_out/envab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
show() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['ms_per_step'],d.get('stage1_ms_per_step'),d.get('stage2_ms_per_step'),d['sampler']['ms_per_batch'])"; }
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-roofline --no-config0 --no-cpu-baseline > gpurun_out/envab/a.log 2>&1 || { tail -5 gpurun_out/envab/a.log; exit 1; }
  echo "base $(show gpurun_out/envab/a.log)"
  env $ABENV timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-roofline --no-config0 --no-cpu-baseline > gpurun_out/envab/b.log 2>&1 || { tail -5 gpurun_out/envab/b.log; exit 1; }
  echo "$ABENV $(show gpurun_out/envab/b.log)"
done

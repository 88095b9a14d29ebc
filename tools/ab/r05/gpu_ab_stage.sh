#!/bin/bash
# A/B of environment switches with the per-stage legs (R5AB="ENV=val;..."), 3 pairs.
set -o pipefail
mkdir -p gpurun_out/abs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
IFS=';' read -ra VARS <<< "$R5AB"
show() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['ms_per_step'],d.get('stage1_ms_per_step'),d.get('stage2_ms_per_step'))"; }
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 $STEPARGS > gpurun_out/abs/base.log 2>&1 || { tail -5 gpurun_out/abs/base.log; exit 1; }
  echo "base $(show gpurun_out/abs/base.log)"
  for v in "${VARS[@]}"; do
    timeout -k 10 200 env $v python bench.py --steps 40 --warmup 5 $STEPARGS > gpurun_out/abs/var.log 2>&1 || { tail -5 gpurun_out/abs/var.log; exit 1; }
    echo "$v $(show gpurun_out/abs/var.log)"
  done
done

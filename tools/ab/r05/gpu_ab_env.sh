#!/bin/bash
# A/B of environment switches on the step-only bench: alternates default / each variant
# (R5AB="ENV=val;ENV2=val2"), 3 pairs.
set -o pipefail
mkdir -p gpurun_out/ab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs"
IFS=';' read -ra VARS <<< "$R5AB"
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 $STEPARGS > gpurun_out/ab/base.log 2>&1 || { tail -5 gpurun_out/ab/base.log; exit 1; }
  echo "base $(python -c "import json;print(json.loads(open('gpurun_out/ab/base.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  for v in "${VARS[@]}"; do
    timeout -k 10 200 env $v python bench.py --steps 40 --warmup 5 $STEPARGS > gpurun_out/ab/var.log 2>&1 || { tail -5 gpurun_out/ab/var.log; exit 1; }
    echo "$v $(python -c "import json;print(json.loads(open('gpurun_out/ab/var.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done

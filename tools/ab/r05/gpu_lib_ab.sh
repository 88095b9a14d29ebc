#!/bin/bash
# A/B of variant libraries ($ALTS, .so paths): isolated roofline leg $LEG per library, then
# the joint step alternated 3 times (tools/gpu_ab_lib.sh).
set -o pipefail
mkdir -p gpurun_out/lab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in default $ALTS; do
  if [ "$lib" = default ]; then E=""; else E="TVQ_HIP_LIB=$lib"; fi
  env $E timeout -k 10 120 python tools/roofline_only.py ${LEG:-wgrad} > gpurun_out/lab/leg.log 2>&1 || { tail -5 gpurun_out/lab/leg.log; exit 1; }
  echo "$(basename $lib) leg $(python -c "import json;d=json.loads(open('gpurun_out/lab/leg.log').read().strip().splitlines()[-1]);print(d['avg_launch_us'], d['frac'])")"
done
bash tools/gpu_ab_lib.sh

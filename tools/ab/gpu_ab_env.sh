#!/bin/bash
# A/B of the joint step between the default and the env settings in $ENVS (";"-separated
# "K=V K2=V2" groups), alternated 3 times.  $PRE (optional): a pytest selection run first.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$PRE" ]; then
  timeout -k 10 600 python -u -m pytest $PRE -x -q --timeout 180 --timeout-method thread > gpurun_out/pre_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/pre_tests.log; [ $rc -eq 0 ] || exit $rc
fi
B="python bench.py --steps 50 --warmup 10 --no-sampler --no-roofline --no-config0 --no-cpu-baseline"
IFS=';' read -ra ALT <<< "$ENVS"
for i in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/abe_def_$i.log 2>&1 || { tail -20 gpurun_out/abe_def_$i.log; exit 1; }
  echo "default $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abe_def_$i.log)"
  k=0
  for e in "${ALT[@]}"; do
    k=$((k+1))
    env $e timeout -k 10 300 $B > gpurun_out/abe_alt${k}_$i.log 2>&1 || { tail -20 gpurun_out/abe_alt${k}_$i.log; exit 1; }
    echo "[$e] $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abe_alt${k}_$i.log)"
  done
done

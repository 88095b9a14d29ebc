#!/bin/bash
# conv_t32 K-stage depth A/B: roofline op alone, then the joint step, per TVQ_CONV_CONFIG
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in ${CONFIGS:-3 19 35}; do
  TVQ_CONV_CONFIG=$c timeout -k 10 120 python tools/roofline_only.py > gpurun_out/t32_$c.log 2>&1 || exit 1
  echo "config $c roofline: $(tail -1 gpurun_out/t32_$c.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["avg_launch_ms"], d["frac"])')"
  TVQ_CONV_CONFIG=$c timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --no-sampler > gpurun_out/t32b_$c.log 2>&1 || exit 1
  echo "config $c bench: $(tail -1 gpurun_out/t32b_$c.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done

#!/bin/bash
# conv_wgrad_w8 staged pipeline: its tests, the wgrad leg alone, then 3 joint-step runs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resblock.py tests/test_fullsize_parity.py tests/test_ops_gpu.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/w8pipe_tests.log 2>&1 || { tail -30 gpurun_out/w8pipe_tests.log; exit 1; }
tail -2 gpurun_out/w8pipe_tests.log
timeout -k 10 120 python tools/roofline_only.py wgrad > gpurun_out/w8pipe_leg.log 2>&1 || { tail -5 gpurun_out/w8pipe_leg.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/w8pipe_leg.log').read().strip().splitlines()[-1]);print('wgrad leg', d['avg_launch_us'], d['frac'])"
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 $STEPARGS > gpurun_out/w8pipe_b.log 2>&1 || { tail -5 gpurun_out/w8pipe_b.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/w8pipe_b.log').read().strip().splitlines()[-1]);print(d['ms_per_step'],d.get('stage1_ms_per_step'),d.get('stage2_ms_per_step'))"
done

#!/bin/bash
# narrow-row norm kernels: their tests + the prior / sampler suites, then the sampler batch
# twice (default library vs $ALT, the previous build) with the joint step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest ${R5T:-tests/test_resblock.py tests/test_sampler_full.py tests/test_sampler.py} \
  -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/norm_tests.log 2>&1 || { tail -30 gpurun_out/norm_tests.log; exit 1; }
tail -2 gpurun_out/norm_tests.log
A="--steps 10 --warmup 3 --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs"
for rep in 1 2; do
  for lib in default $ALT; do
    if [ "$lib" = default ]; then E=""; else E="TVQ_HIP_LIB=$lib"; fi
    env $E timeout -k 10 300 python bench.py $A > gpurun_out/norm_b.log 2>&1 || { tail -5 gpurun_out/norm_b.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/norm_b.log').read().strip().splitlines()[-1]);s=d.get('sampler',{});print('$(basename $lib)', d['ms_per_step'], s.get('ms_per_batch'))"
  done
done

#!/bin/bash
# A/B of LF-prior kernel variants ($ALTS: lib_ab names): correctness (test_prior_eval) and the
# graphed 1024-trajectory sampler batch, alternated.
set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/t-vq-vae-trajgen_amd/lib_ab
for v in $ALTS; do
  TVQ_HIP_LIB=$L/libtvq_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_prior_eval.py tests/test_sampler_full.py > gpurun_out/r6/prior_t_$v.log 2>&1 || { tail -15 gpurun_out/r6/prior_t_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/r6/prior_t_$v.log)"
done
for rep in 1 2 3; do
  for v in default $ALTS; do
    if [ $v = default ]; then E="X=1"; else E="TVQ_HIP_LIB=$L/libtvq_hip_$v.so"; fi
    env $E timeout -k 10 120 python tools/sampler_graph_prof.py 20 > gpurun_out/r6/prior_b.log 2>&1 || { tail -5 gpurun_out/r6/prior_b.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/r6/prior_b.log)"
  done
done

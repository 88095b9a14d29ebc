#!/bin/bash
# Fused eval LF prior: parity tests, then the sampler leg fused vs unfused, then the
# sampler kernel table (rocprofv3) of the fused path.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_prior_eval.py tests/test_sampler.py tests/test_sampler_full.py tests/test_stage2_golden.py -x -q --timeout 180 --timeout-method thread > gpurun_out/prior_tests.log 2>&1
rc=$?; tail -4 gpurun_out/prior_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sampler_only.py 10 > gpurun_out/samp_fused.log 2>&1 || { tail -20 gpurun_out/samp_fused.log; exit 1; }
echo "fused   $(tail -1 gpurun_out/samp_fused.log)"
TVQ_PRIOR_FUSED=0 timeout -k 10 300 python tools/sampler_only.py 10 > gpurun_out/samp_unfused.log 2>&1 || { tail -20 gpurun_out/samp_unfused.log; exit 1; }
echo "unfused $(tail -1 gpurun_out/samp_unfused.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_samp -o samp -- python tools/sampler_only.py 3 > gpurun_out/prof_samp.log 2>&1
echo "rocprof rc=$?"

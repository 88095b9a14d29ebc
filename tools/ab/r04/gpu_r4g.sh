#!/bin/bash
# Round 4: DP overlap form, race sampling (fused HF head + LF prior draw), two-wave LF prior:
# GPU suite, smoke, the graphed sampler batch timed (A/B against the one-wave prior and the
# unfused draw) and profiled.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_prior_eval.py tests/test_sampler.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/r4g_t1.log 2>&1 || { tail -60 gpurun_out/r4g_t1.log; exit 1; }
tail -2 gpurun_out/r4g_t1.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --durations=15 \
  --timeout 240 --timeout-method thread > gpurun_out/r4g_tests.log 2>&1 || { tail -60 gpurun_out/r4g_tests.log; exit 1; }
tail -20 gpurun_out/r4g_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4g_smoke.log 2>&1 || { tail -20 gpurun_out/r4g_smoke.log; exit 1; }
tail -1 gpurun_out/r4g_smoke.log
for i in 1 2; do
  timeout -k 10 300 python tools/sampler_graph_prof.py 20 > gpurun_out/r4g_samp_$i.log 2>&1 || { tail -20 gpurun_out/r4g_samp_$i.log; exit 1; }
  echo "new $(tail -1 gpurun_out/r4g_samp_$i.log)"
  TVQ_PRIOR_WAVES=1 timeout -k 10 300 python tools/sampler_graph_prof.py 20 > gpurun_out/r4g_samp1w_$i.log 2>&1 || { tail -20 gpurun_out/r4g_samp1w_$i.log; exit 1; }
  echo "one-wave prior $(tail -1 gpurun_out/r4g_samp1w_$i.log)"
  TVQ_FUSED_SAMPLE=0 timeout -k 10 300 python tools/sampler_graph_prof.py 20 > gpurun_out/r4g_sampnf_$i.log 2>&1 || { tail -20 gpurun_out/r4g_sampnf_$i.log; exit 1; }
  echo "unfused draw $(tail -1 gpurun_out/r4g_sampnf_$i.log)"
done
rm -rf gpurun_out/r4g_sprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4g_sprof -o samp -- python tools/sampler_graph_prof.py 5 > gpurun_out/r4g_sprof.log 2>&1 || { tail -20 gpurun_out/r4g_sprof.log; exit 1; }
S=$(find gpurun_out/r4g_sprof -name "*kernel_stats.csv" | head -1)
grep -E "maskgit_sample|prior_|gemm_skinny|tied_logits|tls_pack|conv_pack" "$S"

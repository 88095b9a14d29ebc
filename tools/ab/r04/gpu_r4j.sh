#!/bin/bash
# Round 4: cheaper race noise (lowbias32, raw log2, templated tiles): sampling tests, the
# graphed sampler batch timed with the one- and two-wave LF prior, kernel stats.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_prior_eval.py tests/test_sampler.py tests/test_sampler_full.py -x -q -m gpu \
  --timeout 200 --timeout-method thread > gpurun_out/r4j_t1.log 2>&1 || { tail -60 gpurun_out/r4j_t1.log; exit 1; }
tail -2 gpurun_out/r4j_t1.log
for i in 1 2; do
  for V in 1 2; do
    TVQ_PRIOR_WAVES=$V timeout -k 10 300 python tools/sampler_graph_prof.py 20 > gpurun_out/r4j_samp_w${V}_$i.log 2>&1 || { tail -20 gpurun_out/r4j_samp_w${V}_$i.log; exit 1; }
    echo "waves=$V $(tail -1 gpurun_out/r4j_samp_w${V}_$i.log)"
  done
done
for V in 1 2; do
  rm -rf gpurun_out/r4j_sprof_w$V
  TVQ_PRIOR_WAVES=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4j_sprof_w$V -o samp -- python tools/sampler_graph_prof.py 5 > gpurun_out/r4j_sprof_w$V.log 2>&1 || { tail -20 gpurun_out/r4j_sprof_w$V.log; exit 1; }
  S=$(find gpurun_out/r4j_sprof_w$V -name "*kernel_stats.csv" | head -1)
  grep -E "prior_lf_eval|tied_logits" "$S" | cut -d, -f1-5
done

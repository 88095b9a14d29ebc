#!/bin/bash
# tvq_embedding_bwd microbench, then its kernel table under rocprofv3
set -o pipefail
mkdir -p gpurun_out/emb
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python tools/emb_bwd_bench.py > gpurun_out/emb/bench.txt 2>&1 || { cat gpurun_out/emb/bench.txt; exit 1; }
cat gpurun_out/emb/bench.txt
rm -rf gpurun_out/emb/prof
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/emb/prof -o e -- python tools/emb_bwd_bench.py > gpurun_out/emb/prof.log 2>&1 || { tail -20 gpurun_out/emb/prof.log; exit 1; }
S=$(find gpurun_out/emb/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$S" | head -20
find gpurun_out/emb/prof -name "*kernel_trace.csv" -delete

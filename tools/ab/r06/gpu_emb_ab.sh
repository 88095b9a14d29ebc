#!/bin/bash
# tvq_embedding_bwd microbench: lib_ab (base) vs in-tree, alternated
set -o pipefail
mkdir -p gpurun_out/emb
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  echo base; TVQ_HIP_LIB=$GRAFT_REPO_ROOT/lib_ab/libtvq_hip.so timeout -k 10 120 python tools/emb_bwd_bench.py 2>&1 | grep us/call || exit 1
  echo new; timeout -k 10 120 python tools/emb_bwd_bench.py 2>&1 | grep us/call || exit 1
done

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/fb
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python tools/fused_bench.py > gpurun_out/fb/fb.log 2>&1 || { tail -20 gpurun_out/fb/fb.log; exit 1; }
tail -1 gpurun_out/fb/fb.log

#!/bin/bash
# Fused ResBlock phase timing (RB_TIMING build), then the roofline counter legs of the
# step's top kernel (rbbwd) and of the LF 64-channel weight gradient (wgrad).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python tools/rb_timing.py > gpurun_out/rb_timing.txt 2>&1 || { tail -20 gpurun_out/rb_timing.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/rb_timing.txt
LEG=rbbwd bash tools/gpu_roofline.sh && LEG=wgrad bash tools/gpu_roofline.sh

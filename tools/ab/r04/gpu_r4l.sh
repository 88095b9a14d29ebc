#!/bin/bash
# PyTorch-native ops recorded while capturing the joint step graph (warmups included).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/aten_sources.py capture > gpurun_out/r4l_aten_capture.txt 2>&1 || { tail -20 gpurun_out/r4l_aten_capture.txt; exit 1; }
grep -v "Warning\|scheduler.step\|amdgpu.ids" gpurun_out/r4l_aten_capture.txt | grep -v record_stream | head -30

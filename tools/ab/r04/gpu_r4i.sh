#!/bin/bash
# Round 4: PyTorch-native ops left in one eager joint step and one eager sampler batch, then
# the LF prior's PMC (tools/ab/r04/gpu_r4h.sh).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/aten_sources.py > gpurun_out/r4i_aten_step.txt 2>&1 || { tail -20 gpurun_out/r4i_aten_step.txt; exit 1; }
cat gpurun_out/r4i_aten_step.txt | tail -40
timeout -k 10 300 python tools/aten_sources.py sampler > gpurun_out/r4i_aten_sampler.txt 2>&1 || { tail -20 gpurun_out/r4i_aten_sampler.txt; exit 1; }
cat gpurun_out/r4i_aten_sampler.txt | tail -30
bash tools/ab/r04/gpu_r4h.sh

#!/bin/bash
# step kernel table + timeline, then the ResBlock-backward roofline leg's stats and PMC passes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step_prof.sh > gpurun_out/step_prof_out.txt 2>&1 || { tail -20 gpurun_out/step_prof_out.txt; exit 1; }
head -8 gpurun_out/step_prof_out.txt
LEG=rbbwd bash tools/gpu_roofline.sh > gpurun_out/roof_rbbwd.txt 2>&1 || { tail -20 gpurun_out/roof_rbbwd.txt; exit 1; }
tail -3 gpurun_out/roof_rbbwd.txt

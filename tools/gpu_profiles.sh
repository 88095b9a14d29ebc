#!/bin/bash
# Profiles for the bench's roofline object: step-only kernel table, then the PMC evidence
# of the top-time kernel (LEG=wgrad) and of the grouped Linear weight gradients (dominant).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step_prof.sh > gpurun_out/step_prof_out.txt 2>&1 || { tail -20 gpurun_out/step_prof_out.txt; exit 1; }
grep "launches/step" gpurun_out/step_prof_out.txt
LEG=wgrad bash tools/gpu_roofline.sh > gpurun_out/roof_wgrad.txt 2>&1 || { tail -20 gpurun_out/roof_wgrad.txt; exit 1; }
LEG=dominant bash tools/gpu_roofline.sh > gpurun_out/roof_dom.txt 2>&1 || { tail -20 gpurun_out/roof_dom.txt; exit 1; }
echo profiles-done

#!/bin/bash
# Stage1 band chains alone (tools/band_bench.py) + a kernel trace of the LF band.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python tools/band_bench.py > gpurun_out/band.txt 2>&1 || { tail -20 gpurun_out/band.txt; exit 1; }
cat gpurun_out/band.txt | grep -v amdgpu.ids
rm -rf gpurun_out/prof_lf
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_lf -o lf -- python tools/band_bench.py LF > gpurun_out/prof_lf.log 2>&1 || { tail -20 gpurun_out/prof_lf.log; exit 1; }
ls gpurun_out/prof_lf

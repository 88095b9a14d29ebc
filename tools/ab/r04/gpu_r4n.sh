#!/bin/bash
# sampler batch kernel table on the current tree
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/r4n_samp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4n_samp -o samp -- python tools/sampler_graph_prof.py 5 > gpurun_out/r4n_samp.log 2>&1 || { tail -20 gpurun_out/r4n_samp.log; exit 1; }
T=$(find gpurun_out/r4n_samp -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r4n_sampler_batch.csv add_i64_kernel | head -16

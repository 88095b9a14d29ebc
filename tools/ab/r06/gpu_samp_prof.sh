#!/bin/bash
# the sampler batch's kernel table (rocprofv3 over graph-replayed batches)
set -o pipefail
mkdir -p gpurun_out/r6sp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/r6sp/samp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6sp/samp -o samp -- python tools/sampler_graph_prof.py 5 > gpurun_out/r6sp/samp.log 2>&1 || { tail -20 gpurun_out/r6sp/samp.log; exit 1; }
T=$(find gpurun_out/r6sp/samp -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r6sp/sampler_batch_kernels.csv add_i64_kernel > gpurun_out/r6sp/table.txt
python tools/batch_seq.py "$T" add_i64_kernel gpurun_out/r6sp/seq.txt > gpurun_out/r6sp/timeline.txt
rm -f "$T"
head -30 gpurun_out/r6sp/table.txt

#!/bin/bash
# SQ counters of the sampler batch's kernels (one --pmc pass over graph-replayed batches)
set -o pipefail
mkdir -p gpurun_out/r6pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/r6pmc/sq
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES --output-format csv -d gpurun_out/r6pmc/sq -o s -- python tools/sampler_graph_prof.py 2 > gpurun_out/r6pmc/sq.log 2>&1 || { tail -5 gpurun_out/r6pmc/sq.log; exit 1; }
F=$(find gpurun_out/r6pmc/sq -name "*counter_collection.csv" | head -1)
python tools/pmc_kernels.py "$F" > gpurun_out/r6pmc/sq_table.txt; rm -f "$F"
head -40 gpurun_out/r6pmc/sq_table.txt

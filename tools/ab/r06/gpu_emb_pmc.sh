#!/bin/bash
# SQ counters of tvq_embedding_bwd's kernels (tools/emb_bwd_bench.py), one --pmc pass
set -o pipefail
mkdir -p gpurun_out/emb
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/emb/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES --output-format csv -d gpurun_out/emb/pmc -o e -- python tools/emb_bwd_bench.py > gpurun_out/emb/pmc.log 2>&1 || { tail -5 gpurun_out/emb/pmc.log; exit 1; }
F=$(find gpurun_out/emb/pmc -name "*counter_collection.csv" | head -1)
python tools/pmc_kernels.py "$F" "gb_\|seg_" > gpurun_out/emb/pmc_table.txt || true
python tools/pmc_kernels.py "$F" > gpurun_out/emb/pmc_table.txt
rm -f "$F"
cat gpurun_out/emb/pmc_table.txt

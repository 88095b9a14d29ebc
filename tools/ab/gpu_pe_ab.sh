#!/bin/bash
# Fused prior: graphed sampler batch default vs variant libs ($ALTS), then SQ counters of
# the prior kernel (one --pmc pass).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  echo "default $(timeout -k 10 200 python tools/sampler_graph_prof.py 10 2>/dev/null | tail -1)"
  for a in $ALTS; do echo "$(basename $a) $(TVQ_HIP_LIB=$a timeout -k 10 200 python tools/sampler_graph_prof.py 10 2>/dev/null | tail -1)"; done
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM --output-format csv -d gpurun_out/pe_sq -o pe -- python tools/sampler_graph_prof.py 2 > gpurun_out/pe_sq.log 2>&1
echo "pmc rc=$?"

#!/bin/bash
# SQ stall breakdown of the roofline op (conv_t32) per K-stage depth config
mkdir -p gpurun_out/t32pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in ${CONFIGS:-3 19}; do
  TVQ_CONV_CONFIG=$c timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d gpurun_out/t32pmc/c$c -o r -- python tools/roofline_only.py > gpurun_out/t32pmc/c$c.log 2>&1 || exit 1
  TVQ_CONV_CONFIG=$c timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/t32pmc/d$c -o r -- python tools/roofline_only.py > gpurun_out/t32pmc/d$c.log 2>&1 || exit 1
done
echo pmc-done

#!/bin/bash
# PMC passes (one counter group per run) over single conv ops: SHAPE OP pairs in $CASES
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
for c in ${CASES:-"10:fwd"}; do
  si=${c%%:*}; op=${c##*:}
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/t_${si}_${op} -o run -- python tools/conv_one.py $si $op 20 > /dev/null 2>&1 || exit 1
  g=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"; do
    g=$((g+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/p_${si}_${op}_$g -o run -- python tools/conv_one.py $si $op 20 > gpurun_out/pmc/p_${si}_${op}_$g.log 2>&1 || echo "pmc group $g failed for $c"
  done
done
echo done

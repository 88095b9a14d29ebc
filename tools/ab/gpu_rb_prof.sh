#!/bin/bash
# rocprofv3 kernel stats + one SQ counter pass of tools/resblock_bench.py (fused ResBlock)
O=gpurun_out/rbprof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o rb -- python tools/resblock_bench.py > $O/stats.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --output-format csv -d $O/sq -o rb -- python tools/resblock_bench.py > $O/sq.log 2>&1 || exit 1
echo done

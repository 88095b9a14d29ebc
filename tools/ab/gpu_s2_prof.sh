#!/bin/bash
# Kernel durations and L2 traffic of the stride-2 small-channel conv shapes
set -o pipefail
mkdir -p gpurun_out/s2prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2prof
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o s2 -- python tools/conv_shapes_bench.py 3,19,21 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o s2 -- python tools/conv_shapes_bench.py 3,19,21 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $O/pmc2 -o s2 -- python tools/conv_shapes_bench.py 3,19,21 > $O/pmc2.log 2>&1 || { tail -20 $O/pmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw -o s2 -- python tools/conv_shapes_bench.py 3,19,21 > $O/pmcw.log 2>&1 || { tail -20 $O/pmcw.log; exit 1; }
find $O -name "*.csv" | head -20

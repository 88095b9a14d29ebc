#!/bin/bash
# Dominant-kernel evidence for bench.py's roofline object: kernel stats of the roofline op
# alone, then one --pmc pass per counter group (FETCH_SIZE, WRITE_SIZE, MFMA busy).
# Outputs under gpurun_out/roof/.  Each GPU step is time-limited; stop at first failure.
mkdir -p gpurun_out/roof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/roof/stats -o roof -- python tools/roofline_only.py > gpurun_out/roof/stats.log 2>&1 || exit 1
tail -1 gpurun_out/roof/stats.log
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/roof/fetch -o roof -- python tools/roofline_only.py > gpurun_out/roof/fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/roof/write -o roof -- python tools/roofline_only.py > gpurun_out/roof/write.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d gpurun_out/roof/sq -o roof -- python tools/roofline_only.py > gpurun_out/roof/sq.log 2>&1 || exit 1
echo roofline-done

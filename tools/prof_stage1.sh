#!/bin/bash
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/stage1_bench.py --steps 20 > gpurun_out/s1_bench.log 2>&1
cat gpurun_out/s1_bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s1 -o s1 -- python tools/stage1_bench.py --steps 5 --warmup 2 > gpurun_out/prof_s1.log 2>&1
find gpurun_out/prof_s1 -name "*kernel_stats.csv" | head -3

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python tools/ab/r06/cpu_probe.py 16 32 64 2>&1 | tee gpurun_out/r6/cpu_probe.log
TVQ_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-roofline --no-config0 --no-cpu-baseline --no-stage-legs > gpurun_out/r6/bench2.log 2>&1 || { tail -20 gpurun_out/r6/bench2.log; exit 1; }
tail -c 600 gpurun_out/r6/bench2.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-config0 > gpurun_out/r6/bench.log 2>&1 || { tail -20 gpurun_out/r6/bench.log; exit 1; }
tail -c 300 gpurun_out/r6/bench.log

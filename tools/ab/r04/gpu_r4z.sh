#!/bin/bash
# rehearsal of bench.py's N = 2 path (two ranks on cuda:0 over gloo, BranchStepGraph + exchanges)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TVQ_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-sampler --no-roofline --no-config0 --no-cpu-baseline > gpurun_out/r4z_bench2.log 2>&1 || { tail -30 gpurun_out/r4z_bench2.log; exit 1; }
grep "^{" gpurun_out/r4z_bench2.log | cut -c1-400

#!/bin/bash
# sampler (BASELINE config 5): throughput at batch 1024 + kernel stats
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/sampler_bench.py 1024 5 > gpurun_out/sampler.log 2>&1
rc=$?; cat gpurun_out/sampler.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_samp -o samp -- python tools/sampler_bench.py 1024 2 > gpurun_out/prof_samp.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc

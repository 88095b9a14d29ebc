#!/bin/bash
# Sampler batch (configs[4]) time + rocprofv3 kernel table, and one SQ PMC pass over a few
# joint steps (LDS bank conflicts / MFMA of the attention and GEMM kernels).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/sampler_bench.py 1024 5 > gpurun_out/sampler.log 2>&1 || { tail -5 gpurun_out/sampler.log; exit 1; }
tail -1 gpurun_out/sampler.log | cut -c1-300
rm -rf gpurun_out/prof_samp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_samp -o samp -- python tools/sampler_bench.py 1024 2 > gpurun_out/prof_samp.log 2>&1 || { tail -5 gpurun_out/prof_samp.log; exit 1; }
rm -rf gpurun_out/pmc_step
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_step -o step -- python bench.py --steps 3 --warmup 1 --eager --no-sampler --no-roofline --no-config0 --no-cpu-baseline > gpurun_out/pmc_step.log 2>&1 || { tail -5 gpurun_out/pmc_step.log; exit 1; }
echo done

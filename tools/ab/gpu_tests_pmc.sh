#!/bin/bash
# Every -m gpu test, a step-only bench, and one SQ PMC pass over 3 eager joint steps.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -m3 -B5 -A25 "Error\|assert " gpurun_out/pytest_gpu.log | head -80; exit $rc; }
A="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
timeout -k 10 300 python bench.py --steps 30 --warmup 5 $A > gpurun_out/bench_step.log 2>&1 || { tail -20 gpurun_out/bench_step.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_step.log
rm -rf gpurun_out/pmc_step
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_step -o step -- python bench.py --steps 3 --warmup 1 --eager $A > gpurun_out/pmc_step.log 2>&1 || { tail -5 gpurun_out/pmc_step.log; exit 1; }
echo pmc-done

#!/bin/bash
# Copy tools/gpu_r6_evidence.sh's outputs (gpurun_out/, scratch) into profiles/ (tracked).
set -e
cd "$(dirname "$0")/.."
for L in dominant wgrad rbbwd rb32bwd vqassign linfwd t32 attn n16 rb64; do
  cp gpurun_out/roof_$L/traffic.json profiles/r06_${L}_traffic.json
  cp gpurun_out/roof_$L/stats/roof_kernel_stats.csv profiles/r06_${L}_kernel_stats.csv
done
cp gpurun_out/r6ev/step_kernel_stats.csv profiles/r06_step_kernel_stats.csv
cp gpurun_out/r6ev/sampler_batch_kernels.csv profiles/r06_sampler_batch_kernels.csv
cp gpurun_out/r6ev/step_timeline.txt profiles/r06_step_timeline.txt
cp gpurun_out/r6ev/step_table.txt profiles/r06_step_table.txt
cp gpurun_out/r6ev/bench.log profiles/r06_bench_full.log; tail -1 gpurun_out/r6ev/bench.log > profiles/r06_bench.json; tail -3 gpurun_out/r6ev/pytest_gpu.log > profiles/r06_gpu_tests_tail.txt; tail -4 gpurun_out/r6ev/smoke.log >> profiles/r06_gpu_tests_tail.txt

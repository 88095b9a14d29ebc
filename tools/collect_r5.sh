#!/bin/bash
# Copy tools/gpu_r5_evidence.sh's outputs (gpurun_out/, scratch) into profiles/ (tracked).
set -e
cd "$(dirname "$0")/.."
for L in dominant wgrad rbbwd vqassign linfwd t32 attn n16 rb64; do
  cp gpurun_out/roof_$L/traffic.json profiles/r05_${L}_traffic.json
  cp gpurun_out/roof_$L/stats/roof_kernel_stats.csv profiles/r05_${L}_kernel_stats.csv
done
cp gpurun_out/r5ev/step_kernel_stats.csv profiles/r05_step_kernel_stats.csv
cp gpurun_out/r5ev/sampler_batch_kernels.csv profiles/r05_sampler_batch_kernels.csv
cp gpurun_out/r5ev/step_timeline.txt profiles/r05_step_timeline.txt
cp gpurun_out/r5ev/step_table.txt profiles/r05_step_table.txt

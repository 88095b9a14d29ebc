#!/bin/bash
# Step time under conv engine configurations (TVQ_CONV_CONFIG bits, tvq_conv_config).
mkdir -p gpurun_out
A="--no-sampler --no-roofline --no-config0 --no-cpu-baseline --steps 30 --warmup 5"
for C in 3 11 19 35 3; do
  TVQ_CONV_CONFIG=$C timeout -k 10 200 python bench.py $A > gpurun_out/cfg.log 2>&1 || { tail -5 gpurun_out/cfg.log; exit 1; }
  echo "conv_config=$C $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/cfg.log)"
done

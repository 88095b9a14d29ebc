#!/bin/bash
A="--no-sampler --no-roofline --no-config0 --no-cpu-baseline --steps 30 --warmup 5"
mkdir -p gpurun_out
for O in "" grad "grad,vq"; do
  TVQ_STREAMS_OFFLOAD="$O" timeout -k 10 200 python bench.py $A > gpurun_out/offl.log 2>&1
  rc=$?
  echo "offload=[$O] rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/offl.log)"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/offl.log; exit 1; }
done

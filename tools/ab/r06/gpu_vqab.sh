#!/bin/bash
# vq_assign variants (double-buffered codebook chunks, LF row groups): parity of each library
# build, the assign kernel's time under rocprofv3, then joint-step A/B against the in-tree build
set -o pipefail
mkdir -p gpurun_out/vqab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in 0 1 2 3; do
  if [ $n = 0 ]; then unset TVQ_HIP_LIB; else export TVQ_HIP_LIB=$GRAFT_REPO_ROOT/lib_ab$n/libtvq_hip.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_vq.py tests/test_fullsize_parity.py -q -m gpu -k "vq or VQ or stage1" --timeout 120 --timeout-method thread > gpurun_out/vqab/t$n.log 2>&1 || { tail -30 gpurun_out/vqab/t$n.log; exit 1; }
  echo "lib$n tests: $(tail -1 gpurun_out/vqab/t$n.log)"
  rm -rf gpurun_out/vqab/p$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vqab/p$n -o p -- python tools/vq_microbench.py > gpurun_out/vqab/m$n.log 2>&1 || { tail -20 gpurun_out/vqab/m$n.log; exit 1; }
  S=$(find gpurun_out/vqab/p$n -name "*kernel_stats.csv" | head -1)
  grep vq_assign "$S" | cut -d, -f1-5 | sed "s/^/lib$n /"
  find gpurun_out/vqab/p$n -name "*kernel_trace.csv" -delete
done
unset TVQ_HIP_LIB
show() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['ms_per_step'],d.get('stage1_ms_per_step'),d.get('stage2_ms_per_step'))"; }
for rep in 1 2; do
  for n in 0 ${VQAB_LIBS:-1 3}; do
    if [ $n = 0 ]; then unset TVQ_HIP_LIB; else export TVQ_HIP_LIB=$GRAFT_REPO_ROOT/lib_ab$n/libtvq_hip.so; fi
    timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-roofline --no-config0 --no-cpu-baseline --no-sampler > gpurun_out/vqab/b$n.log 2>&1 || { tail -5 gpurun_out/vqab/b$n.log; exit 1; }
    echo "lib$n $(show gpurun_out/vqab/b$n.log)"
  done
done

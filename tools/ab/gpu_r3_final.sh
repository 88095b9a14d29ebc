#!/bin/bash
# Round-3 evidence on one tree: every -m gpu test, smoke(), the full bench line, the step's
# kernel table / timeline, the roofline legs' PMC passes (LEG list), the sampler graph's
# kernel table.  Each GPU step time-limited; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
grep "smoke ok" gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log > gpurun_out/bench_full.json
echo bench-done
bash tools/gpu_evidence.sh > gpurun_out/evidence.txt 2>&1 || { tail -20 gpurun_out/evidence.txt; exit 1; }
head -6 gpurun_out/evidence.txt
for L in ${LEGS:-linfwd}; do
  LEG=$L bash tools/gpu_roofline.sh > gpurun_out/roof_$L.txt 2>&1 || { tail -20 gpurun_out/roof_$L.txt; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sgraph -o sg -- python tools/sampler_graph_prof.py > gpurun_out/prof_sgraph.log 2>&1 || { tail -20 gpurun_out/prof_sgraph.log; exit 1; }
echo r3-final-done

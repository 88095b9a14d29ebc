#!/bin/bash
# Round 5: the C = 64 fused ResBlock -- its tests, the full-size parity and stage tests, the
# step bench with the per-stage legs and a step kernel table.
set -o pipefail
mkdir -p gpurun_out/r5b
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_resblock.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/r5b/t_rb.log 2>&1
rc=$?; tail -15 gpurun_out/r5b/t_rb.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_fullsize_parity.py tests/test_stage1.py tests/test_stage2_golden.py tests/test_graph.py tests/test_fused_ff.py -q -m gpu -x -rP --timeout 180 --timeout-method thread > gpurun_out/r5b/t_full.log 2>&1
rc=$?; tail -3 gpurun_out/r5b/t_full.log; grep "flips=" gpurun_out/r5b/t_full.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/r5b/t_full.log | tail -60; exit $rc; }
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > gpurun_out/r5b/bench_step.log 2>&1 || { tail -20 gpurun_out/r5b/bench_step.log; exit 1; }
tail -1 gpurun_out/r5b/bench_step.log | cut -c1-300
python -c "import json;d=json.loads(open('gpurun_out/r5b/bench_step.log').read().strip().splitlines()[-1]);print('ms',d['ms_per_step'],'s1',d.get('stage1_ms_per_step'),'s2',d.get('stage2_ms_per_step'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5b/prof -o step -- python bench.py --steps 5 --warmup 2 --no-stage-legs $STEPARGS > gpurun_out/r5b/prof.log 2>&1 || { tail -20 gpurun_out/r5b/prof.log; exit 1; }
T=$(find gpurun_out/r5b/prof -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 gpurun_out/r5b/step_table.csv > gpurun_out/r5b/step_table.txt
python tools/step_timeline.py "$T" 2 12 > gpurun_out/r5b/step_timeline.txt
head -3 gpurun_out/r5b/step_table.txt
rm -f "$T"
echo r5b-done

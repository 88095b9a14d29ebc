#!/bin/bash
# Round 5 iteration: resblock tests, step bench with per-stage legs, step kernel table.
set -o pipefail
D=gpurun_out/${R5TAG:-r5c}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest ${R5TESTS:-tests/test_resblock.py} -q -m gpu -x --timeout 120 --timeout-method thread > $D/t.log 2>&1
rc=$?; tail -3 $D/t.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $D/t.log | tail -60; exit $rc; }
STEPARGS="--no-sampler --no-roofline --no-config0 --no-cpu-baseline"
timeout -k 10 300 python bench.py --steps 30 --warmup 5 $STEPARGS > $D/bench_step.log 2>&1 || { tail -20 $D/bench_step.log; exit 1; }
python -c "import json;d=json.loads(open('$D/bench_step.log').read().strip().splitlines()[-1]);print('ms',d['ms_per_step'],'s1',d.get('stage1_ms_per_step'),'s2',d.get('stage2_ms_per_step'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o step -- python bench.py --steps 5 --warmup 2 --no-stage-legs $STEPARGS > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
T=$(find $D/prof -name "*kernel_trace.csv" | head -1)
python tools/step_table.py "$T" 5 $D/step_table.csv > $D/step_table.txt
python tools/step_timeline.py "$T" 2 12 > $D/step_timeline.txt
head -1 $D/step_table.txt
grep -E "${R5GREP:-w8}" $D/step_table.csv || true
rm -f "$T"
echo done

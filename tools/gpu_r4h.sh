#!/bin/bash
# Round 4: PMC of the sampler's LF prior launch (MFMA busy share, wave waits, clock):
# rocprofv3 --pmc passes over 2 graphed sampling batches, prior_lf_eval_kernel only.
set -o pipefail
O=gpurun_out/r4h_prior
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
F="--kernel-include-regex prior_lf_eval"
timeout -s KILL 120 rocprofv3 $F --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/sq -o p -- python tools/sampler_graph_prof.py 2 > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 $F --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d $O/sq2 -o p -- python tools/sampler_graph_prof.py 2 > $O/sq2.log 2>&1 || { tail -5 $O/sq2.log; exit 1; }
for d in sq sq2; do
  f=$(find $O/$d -name "*counter_collection.csv" | head -1)
  python - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k}: n={len(v)} avg={sum(v)/len(v):.4g}")
PY
done

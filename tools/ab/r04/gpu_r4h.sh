#!/bin/bash
# Round 4: PMC of the sampler's LF prior launch, one-wave and two-wave kernels (MFMA busy
# share, wave waits, clock), and of the fused HF head+draw: rocprofv3 --pmc passes over 2
# graphed sampling batches.
set -o pipefail
O=gpurun_out/r4h_prior
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
F="--kernel-include-regex prior_lf_eval|tied_logits_sample"
for V in 2 1; do
  export TVQ_PRIOR_WAVES=$V
  timeout -s KILL 120 rocprofv3 $F --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/sq_w$V -o p -- python tools/sampler_graph_prof.py 2 > $O/sq_w$V.log 2>&1 || { tail -5 $O/sq_w$V.log; exit 1; }
  timeout -s KILL 120 rocprofv3 $F --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d $O/sq2_w$V -o p -- python tools/sampler_graph_prof.py 2 > $O/sq2_w$V.log 2>&1 || { tail -5 $O/sq2_w$V.log; exit 1; }
  for d in sq_w$V sq2_w$V; do
    f=$(find $O/$d -name "*counter_collection.csv" | head -1)
    echo "== $d"
    python - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0][-40:]
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(cs.items())})
PY
  done
done

#!/bin/bash
# GEMM parity tests, then the GEMM micro-bench with the direct kernels off / on (TNW 1, 2, 4).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -m gpu -k "gemm or linear" \
  --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -3 gpurun_out/gemm_tests.log
TVQ_GEMM_LDS=0 timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/gemm_base.log 2>&1 || exit 1
timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/gemm_new.log 2>&1 || exit 1
python - <<'PY'
import json
rows = {}
for tag in ["base", "new"]:
    for l in open(f"gpurun_out/gemm_{tag}.log"):
        if l.startswith("{"):
            r = json.loads(l); rows.setdefault(r["name"], {})[tag] = r["us"]
for k, v in rows.items():
    print(f"{k:22s}", "  ".join(f"{t}={v.get(t)}" for t in ["base", "new"]))
PY

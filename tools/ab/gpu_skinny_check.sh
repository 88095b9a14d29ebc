#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_stage2_golden.py tests/test_sampler.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/skt.log 2>&1 || { tail -30 gpurun_out/skt.log; exit 1; }
tail -1 gpurun_out/skt.log
timeout -k 10 200 python tools/sampler_bench.py 1024 5 --no-cpu-baseline > gpurun_out/rb2s.log 2>&1 || exit 1
tail -1 gpurun_out/rb2s.log | cut -c1-140
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_g -o g -- python tools/gemm_bench.py lf_logits_sampler > gpurun_out/pmc_g.log 2>&1 || exit 1
python - <<'PY'
import csv,collections
agg=collections.defaultdict(lambda: collections.defaultdict(float)); cnt=collections.Counter()
import glob
f=glob.glob('gpurun_out/pmc_g/**/*counter_collection.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    k=r['Kernel_Name'][:50]; agg[k][r['Counter_Name']]+=float(r['Counter_Value'])
    if r['Counter_Name']=='SQ_INSTS_LDS': cnt[k]+=1
for k,v in agg.items():
    if 'skinny' in k: print(k, cnt[k], v['SQ_LDS_BANK_CONFLICT']/cnt[k], v['SQ_INSTS_LDS']/cnt[k])
PY

#!/bin/bash
# marching prolongation: chunk length x prefetch depth (bench fine-kernel table, P0 ms)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
P=gpurun_out/ptune
mkdir -p $P
timeout -k 10 200 python -u -m pytest tests/test_gpu_march.py -q -m gpu -x --timeout 120 --timeout-method thread > $P/pytest.log 2>&1 || exit $?
tail -1 $P/pytest.log
for cfg in "16 1" "16 2" "32 1" "32 2" "8 2" "64 2"; do
  set -- $cfg
  AMG_PROLONG_ZC=$1 AMG_PROLONG_PF=$2 timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 30 > $P/b_$1_$2.json 2> $P/b_$1_$2.log || exit $?
  python -c "
import json,sys
d=json.load(open('$P/b_$1_$2.json')); fk=d.get('fine_kernels',{})
p=fk.get('prolong0'); print('zc $1 pf $2', round(d['value'],1), round(d['ms_per_step'],4), p if not isinstance(p,dict) else {k:p[k] for k in ('ms','frac') if k in p})"
done

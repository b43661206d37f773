#!/bin/bash
# slab V-cycle zero-guess fold: slab/dist tests, one-rank slab bench A/B, then the whole GPU tier
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
P=gpurun_out/slabzg
mkdir -p $P
AMG_ZG_FOLD_SLAB=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_dist.py -q -m gpu -x --timeout 300 --timeout-method thread > $P/pytest_slab.log 2>&1
st=$?; echo "pytest exit $st" >> $P/pytest_slab.log; tail -2 $P/pytest_slab.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python bench.py --gpus 1 --force-dist 1 --cpu-baseline 0 > $P/dist_old.json 2> $P/dist_old.log || exit $?
AMG_ZG_FOLD_SLAB=1 timeout -k 10 300 python bench.py --gpus 1 --force-dist 1 --cpu-baseline 0 > $P/dist_new.json 2> $P/dist_new.log || exit $?
python -c "
import json
for k in ('old','new'):
    d=json.load(open('$P/dist_'+k+'.json')); print(k, round(d['value'],1), round(d['ms_per_step'],4))"
bash tools/gpu_tests_only.sh

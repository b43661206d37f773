#!/bin/bash
# round 5 (y): reciprocal division on the plain-CSR / bsr3 paths: parity, general-CSR A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05y
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solve.py tests/test_gpu_classical.py \
   tests/test_gpu_bsr.py tests/test_gpu_configs.py tests/test_gpu_master.py -m "gpu and not slow" -x -q --timeout 200 \
   --timeout-method thread > $O/tests.log 2>&1; echo "tests exit $?"; tail -1 $O/tests.log
for v in 1 0 1 0; do
  AMG_FAST_DIV=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --steps 10 > $O/g$v.json 2> $O/g$v.err
  echo "fast_div $v: $(python3 -c "import json; d=json.load(open('$O/g$v.json')); g=d['vcycle_general_csr']; print(round(d['ms_per_step'],3), round(g['value'],2), {k: round(v['ms'],3) for k, v in g['fine_kernels'].items()})")"
done

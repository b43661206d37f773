#!/bin/bash
# round 5 (as): the long-row CSR kernel with 128 / 256 rows per workgroup on the
# largest levels (AMG_LONG_RW) -- bitwise tests, then elasticity r = 6 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05as
mkdir -p $O
for rw in 128 256; do
  AMG_LONG_RW=$rw timeout -k 10 300 python -u -m pytest tests/test_gpu_classical.py tests/test_gpu_kernels.py -m "gpu and not slow" -x -q --timeout 200 --timeout-method thread > $O/t$rw.log 2>&1
  rc=$?; echo "tests rw $rw: $(tail -1 $O/t$rw.log)"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for rw in 0 128 256; do
    AMG_LONG_RW=$rw timeout -k 10 400 python -u tools/bench_elasticity.py --refine 6 > $O/e_${rw}_$i.json 2> $O/e_${rw}_$i.err
    rc=$?; [ $rc -eq 0 ] || { echo "elast rw $rw exit $rc"; exit $rc; }
    echo "rw $rw: $(python3 -c "import json; d=json.load(open('$O/e_${rw}_$i.json')); print(round(d['it_per_s'],2), round(d['ms_per_step'],3), 'ms', d['relres_after'])")"
  done
done

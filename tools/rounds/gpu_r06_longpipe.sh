# long-row kernel with the next chunk's streams in flight during the sums (AMG_LONG_PIPE=1):
# the long-row kernel tests under it, then the elasticity r=6 A/B
set -o pipefail
O=${1:-gpurun_out/r06/longpipe}
mkdir -p $O
AMG_LONG_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_classical.py -x -q --timeout 200 --timeout-method thread -k "matvec or residual or jacobi or spgemv or elasticity_solve or classical_solve" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for v in "AMG_LONG_PIPE=0" "AMG_LONG_PIPE=1"; do
  tag=$(echo "$v" | tr ' =' '_-')
  env $v timeout -k 10 400 python3 tools/bench_elasticity.py --refine 6 --steps 20 > $O/e_${tag}_$rep.json 2> $O/e_${tag}_$rep.err || { echo "variant $v failed"; tail -5 $O/e_${tag}_$rep.err; exit 1; }
  python3 - "$v" $O/e_${tag}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"[{sys.argv[1]}] {d['it_per_s']:.1f} it/s {d['ms_per_step']:.3f} ms/step; coarse SpMV:",
      " ".join(f"L{c['level']} {c['per_row']:.0f}/row {c['ms']*1e3:.0f}us {c['frac']:.3f}" for c in d["coarse_spmv"]))
PY
done
done

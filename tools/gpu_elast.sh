# config-5 elasticity bench on one GPU: r = 5 and 6 (3x3 blocks), with the
# classical setup on the host
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for R in ${RS:-5 6}; do
  timeout -k 10 900 python tools/bench_elasticity.py --refine $R --steps 20 > gpurun_out/elast_r$R.json 2> gpurun_out/elast_r$R.log
  st=$?; tail -2 gpurun_out/elast_r$R.log; cat gpurun_out/elast_r$R.json; [ $st -eq 0 ] || exit $st
done

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
tail -4 gpurun_out/pytest_gpu.log
for R in 0 1; do
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --reuse-outer-residual $R > gpurun_out/bench_reuse$R.json 2> gpurun_out/bench_reuse$R.err || exit 1
grep -E "steps in|fine residual" gpurun_out/bench_reuse$R.err
done

# a subset of the GPU suite in one process: ./tools/rounds/gpu_r06_sub.sh OUTDIR pytest-args...
set -o pipefail
O=$1; shift
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -m gpu -s --maxfail=25 --timeout 300 --timeout-method thread "$@" > $O/sub.log 2>&1
rc=$?
echo "sub rc=$rc"
grep -E "OUTSIDE|FAILED|passed|failed|run [0-9]+:" $O/sub.log | tail -60
exit 0

# the whole GPU suite in one process, as the driver runs it (here without -x,
# so every failure shows); -rA summary, per-test durations
set -o pipefail
O=${1:-gpurun_out/r06/suite}
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests/ -q -m gpu -s --maxfail=25 --timeout 300 --timeout-method thread --durations=30 > $O/suite.log 2>&1
rc=$?
echo "suite rc=$rc"
grep -E "OUTSIDE|FAILED|passed|failed" $O/suite.log | tail -40
exit 0

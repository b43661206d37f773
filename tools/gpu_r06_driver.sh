# the driver's GPU tiers on this tree: the whole GPU suite in ONE process with
# -x (as GPUTEST runs it), smoke(), then the default bench line
set -o pipefail
O=${1:-gpurun_out/r06/driver}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gputest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'roof', d['roofline']['frac'], 'csr', d['roofline_csr']['frac'])
c=d['cpu_baseline']; print('cpu', c and c['value'], c and c['cores'], c and c.get('all_cores'))
print('parity', d['parity'])
"

#!/bin/bash
# slab hierarchy tests + 1-rank distributed bench vs single-GPU bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/slab
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_dist.py -v -s --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed|relres" $out/pytest.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --gpus 1 --force-dist 1 --steps 20 --warmup 3 > $out/bench_dist1.json 2> $out/bench_dist1.log || exit $?
echo "dist1: $(python -c "import json;d=json.load(open('$out/bench_dist1.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity'])")"

#!/bin/bash
# round 5 (a): the ADVICE fixes (composed-transfer gating with zero sweeps,
# res GLOBAL + converge GLOBAL round robin) in test_gpu_async.py, the
# process-rank slab async solve (cross-process channels), a 2-process run of
# tools/bench_dist_async.py under torchrun, smoke()
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
export AMG_SEGV_TRACE=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_async.py -v -s -rf --timeout 170 \
   --timeout-method thread > $O/async.log 2>&1
rc=$?; echo "async exit $rc"; grep -E "passed|failed" $O/async.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_slab_async_procs.py -v -s -rf --timeout 300 \
   --timeout-method thread > $O/procs.log 2>&1
rc=$?; echo "procs exit $rc"; grep -E "passed|failed" $O/procs.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
   --master-port=29611 tools/bench_dist_async.py --size 128 --cycles 8 --runs 2 --transport host --rep 4096 \
   > $O/bench_async_procs.json 2> $O/bench_async_procs.err
rc=$?; echo "bench procs exit $rc"; cat $O/bench_async_procs.json | head -c 600
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -2 $O/smoke.log
exit $rc

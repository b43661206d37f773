# The N>1 leg of bench.py as the driver launches it (torchrun, RCCL), at one
# rank: dist GPU tests, the dist bench line, and a kernel trace of it.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/dist1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dist1/pytest_dist.log 2>&1
st=$?; tail -3 gpurun_out/dist1/pytest_dist.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 \
   bench.py --gpus 1 --force-dist 1 --steps 20 --warmup 3 > gpurun_out/dist1/bench.json 2> gpurun_out/dist1/bench.err
st=$?; tail -3 gpurun_out/dist1/bench.err; cat gpurun_out/dist1/bench.json; [ $st -eq 0 ] || exit $st
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/dist1/trace -o run \
   -- python3 $R/bench.py --force-dist 1 --steps 10 --warmup 2 > $R/gpurun_out/dist1/trace_bench.json 2> $R/gpurun_out/dist1/trace_bench.err
st=$?; tail -2 $R/gpurun_out/dist1/trace_bench.err; exit $st

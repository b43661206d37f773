set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
nproc > gpurun_out/host.txt; lscpu | grep -E "Model name|^CPU\(s\)" >> gpurun_out/host.txt; free -g >> gpurun_out/host.txt
timeout -k 10 900 python bench.py --steps 20 --warmup 3 > gpurun_out/bench512.json 2> gpurun_out/bench512.err
echo "bench exit $?"
tail -3 gpurun_out/bench512.err; cat gpurun_out/bench512.json

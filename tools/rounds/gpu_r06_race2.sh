# one-rank distributed async multadd race: default (add, wait, read-back) vs
# the capture form (AMG_ATOMIC_NORET=0), per-row replay of every run
set -o pipefail
mkdir -p gpurun_out/r06
for m in 1 0 1 0; do
  AMG_ATOMIC_NORET=$m AMG_REPLAY_DUMP=gpurun_out/r06/dump2_m$m timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dist.py -k "test_dist_async_band and multadd-cuts3" > gpurun_out/r06/race2_m$m.log 2>&1
  echo "noret=$m rc=$?"
  grep -E "run [0-9]+:" gpurun_out/r06/race2_m$m.log
done
exit 0

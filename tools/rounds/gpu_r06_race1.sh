set -o pipefail
mkdir -p gpurun_out/r06
export AMG_REPLAY_DUMP=gpurun_out/r06/dump1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py -k "async_band or accel" > gpurun_out/r06/race1.log 2>&1
echo rc=$?
grep -E "run [0-9]+:|passed|failed" gpurun_out/r06/race1.log | tail -40

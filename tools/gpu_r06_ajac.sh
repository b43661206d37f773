# DMEM_AsyncSmooth overlap at 512^3, 2 ranks, the box's default hardware
# queues: comm stream at high priority (default) vs normal priority
set -o pipefail
O=gpurun_out/r06/ajac
mkdir -p $O
for p in 1 0 1 0; do
  AMG_COMM_PRIORITY=$p timeout -k 10 240 python -u tools/bench_async_jacobi.py --ranks 2 > $O/ajac_p$p.json 2> $O/ajac_p$p.err || { echo "ajac p=$p failed"; tail -5 $O/ajac_p$p.err; exit 1; }
  echo "prio=$p"; cat $O/ajac_p$p.err | grep rank
done

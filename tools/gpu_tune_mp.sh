# interleaved A/B of the master-pattern kernel forms on the 512^3 operators
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/tune_spmv.py 512 7 mp,ABL_mp > gpurun_out/tune_mp.log 2>&1; st=$?; cat gpurun_out/tune_mp.log; exit $st

# FETCH_SIZE / WRITE_SIZE passes of tools/pmc_run.py 512 under an environment
# setting (ENVSET="AMG_MZ_LINES=2"), reduced by pmc_fine.py into gpurun_out/traffic_env.json
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
P=$R/gpurun_out/pe
rm -rf $P; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
export $ENVSET
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $P/fetch -o run \
   -- python3 $R/tools/pmc_run.py 512 > $P/fetch.log 2>&1 || exit $?
echo "fetch ok"
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $P/write -o run \
   -- python3 $R/tools/pmc_run.py 512 > $P/write.log 2>&1 || exit $?
echo "write ok"
F=$(find $P/fetch -name "*counter_collection.csv" | head -1)
W=$(find $P/write -name "*counter_collection.csv" | head -1)
echo '{}' > $R/gpurun_out/traffic_env.json
cd $R/tools && python3 pmc_fine.py $F $W 512 $R/gpurun_out/traffic_env.json > $R/gpurun_out/pmc_env.log 2>&1
grep -E '^ "|traffic_over_alg' $R/gpurun_out/pmc_env.log

cd $GRAFT_REPO_ROOT
timeout -k 10 600 python tools/tune_spmv.py 512 5

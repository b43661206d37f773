cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/debug_jgs.py

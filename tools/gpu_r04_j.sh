#!/bin/bash
# round 4: the sync slab file after the fix of the out-of-range DLevel write
# (slab_vcycle wrote zero_done one entry past D->lv when restricting into the
# replicated tail): host-checked library and the zero-guess fold on, then the
# normal library (fold on, and the default), then the level-0 variants
set -o pipefail
mkdir -p gpurun_out/r04j
export AMG_SEGV_TRACE=1
run() { # name timeout env... -- pytest args
   local name=$1 t=$2; shift 2
   env "$@" timeout -k 10 $t python -u -m pytest -p no:faulthandler tests/test_gpu_slab.py -k "not 512" -x -v -s -rf \
      --timeout 170 --timeout-method thread > gpurun_out/r04j/$name.log 2>&1
   local rc=$?
   echo "$name exit $rc"; grep -E "passed|failed|Assertion|signal" gpurun_out/r04j/$name.log | tail -3
   [ $rc -eq 0 ] || exit $rc
}
run slab_chk_fold 400 AMG_CHK_LIB=1 MALLOC_CHECK_=3 AMG_ZG_FOLD_SLAB=1
run slab_fold 300 AMG_ZG_FOLD_SLAB=1
run slab_default 300 AMG_ZG_FOLD_SLAB=0
./tools/gpu_r04_h.sh

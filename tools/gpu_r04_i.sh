#!/bin/bash
# round 4: the sync slab file's host heap fault (malloc segfault in the case
# after the first 2-rank case, fold off) under the host-checked library
# (AMG_CHK_LIB=1: bounds-checked std containers) with glibc's heap checks, the
# native backtrace on SEGV / BUS / ABRT; then the level-0 variants
set -o pipefail
mkdir -p gpurun_out/r04i
export AMG_SEGV_TRACE=1
AMG_CHK_LIB=1 MALLOC_CHECK_=3 MALLOC_PERTURB_=165 timeout -k 10 300 python -u -m pytest -p no:faulthandler \
   tests/test_gpu_slab.py -k "not 512" -x -v -s -rf --timeout 170 --timeout-method thread > gpurun_out/r04i/slab_chk.log 2>&1
rc=$?; echo "slab_chk exit $rc"; grep -E "passed|failed|Assertion|signal|malloc|free\(\)" gpurun_out/r04i/slab_chk.log | head -8
[ $rc -eq 0 ] || exit $rc
./tools/gpu_r04_h.sh

#!/bin/bash
# fine SpMV under march variants
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in "" "AMG_MZ_LINES=2" "AMG_PLANE_MARCH=32" "AMG_PLANE_MARCH=64" "AMG_PLANE_MARCH=8" "AMG_MZ_NT=1" "AMG_PLANE_MARCH_XCD=0"; do
  env $v timeout -k 10 120 python tools/spmv_variants.py 512 || exit $?
done

#!/bin/bash
# fine-sweep over-fetch study: FETCH_SIZE and TCC hit/miss of the post-sweep per march variant
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
P=$R/gpurun_out/overfetch
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
if [ $# -eq 0 ]; then
  set -- "default:" "lines2:AMG_MZ_LINES=2" "zc64:AMG_PLANE_MARCH=64" "zc8:AMG_PLANE_MARCH=8" "noxcd:AMG_PLANE_MARCH_XCD=0" "nt0:AMG_MZ_NT=0"
fi
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $P/$name/fetch -o run \
     -- python3 $R/tools/pmc_sweep.py 512 > $P/$name.fetch.log 2>&1 || exit $?
  env $envs timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $P/$name/hit -o run \
     -- python3 $R/tools/pmc_sweep.py 512 > $P/$name.hit.log 2>&1 || exit $?
  echo "$name ok"
done
echo done

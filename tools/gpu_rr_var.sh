#!/bin/bash
# fused residual + restriction variants: bench it/s and the kernel time
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in "" "AMG_RR_LINES=2" "AMG_RR_OCC=5" "AMG_RR_RING=1" "AMG_PLANE_MARCH=32"; do
  env $v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/bench_rr.json 2> gpurun_out/bench_rr.log || exit $?
  echo "${v:-default}: $(python -c "import json;d=json.load(open('gpurun_out/bench_rr.json'));k=d['fine_kernels'];print(round(d['value'],1), round(d['ms_per_step'],3), {n:round(v['ms'],3) for n,v in k.items()})")"
done

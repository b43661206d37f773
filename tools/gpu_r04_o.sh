#!/bin/bash
# interleaved A/B of the 7-pt march defaults on one box: old (prefetch 1,
# mz_chunk's rule) against new (prefetch 2, occupancy-sized chunks), bench.py
# without the CPU leg, twice each
set -o pipefail
mkdir -p gpurun_out/r04o
for i in 1 2; do
  for v in "AMG_MZ_PF=1 AMG_MZ_OCC=0" "AMG_MZ_PF=2 AMG_MZ_OCC=-1"; do
    name=$(echo $v | tr ' =' '__')_$i
    env $v timeout -k 10 240 python -u bench.py --cpu-baseline 0 > gpurun_out/r04o/$name.json 2> gpurun_out/r04o/$name.log
    st=$?; [ $st -eq 0 ] || { echo "$name exit $st"; exit $st; }
    python3 -c "
import json; d=json.load(open('gpurun_out/r04o/$name.json')); k=d['fine_kernels']
print('$name', round(d['value'],1), round(d['ms_per_step'],4), round(k['outer_residual_sweep']['ms'],4), round(k['post_sweep']['ms'],4))"
  done
done

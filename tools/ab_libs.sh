#!/bin/bash
# Alternating bench runs over the product library and diagnostic variants lib/diag/libdgs_<v>.so (kernel timing all)
set -u
for i in $(seq ${RUNS:-2}); do
  for v in product ${VARIANTS:?}; do
    if [ $v = product ]; then unset DGS_LIB; else export DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_$v.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --kernel-timing all > gpurun_out/ab3.log 2>&1 || { tail -5 gpurun_out/ab3.log; exit 1; }
    tail -1 gpurun_out/ab3.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());k=d['kernels_ms_per_step']
print('$v', round(d['value'],1), {a: round(b,4) for a,b in k.items() })"
  done
done

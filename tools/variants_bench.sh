#!/bin/bash
# Alternating bench runs of the product library and diagnostic variants lib/diag/libdgs_<v>.so with
# every kernel class timed; prints steps/s, ms/step and the classes in $CLASSES (default: all)
#   VARIANTS="a b" [ROUNDS=2] [CLASSES="depth_sort,place"] tools/variants_bench.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in $(seq ${ROUNDS:-2}); do
  for v in product ${VARIANTS:?}; do
    if [ $v = product ]; then unset DGS_LIB; else export DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_$v.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-timing all > gpurun_out/vb.log 2>&1 || { tail -5 gpurun_out/vb.log; exit 1; }
    tail -1 gpurun_out/vb.log | CL="${CLASSES:-}" python3 -c "
import json,os,sys;d=json.loads(sys.stdin.read());k=d['kernels_ms_per_step'];cl=[c for c in os.environ['CL'].split(',') if c]
print('$v', round(d['value'],1), round(d['ms_per_step'],3), {a: round(b,4) for a,b in k.items() if not cl or a in cl})"
  done
done

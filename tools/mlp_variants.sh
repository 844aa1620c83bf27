#!/bin/bash
# MLP kernel times (tools/mlp_time.py, split arithmetic) for the product library and diagnostic
# variants lib/diag/libdgs_<v>.so:  VARIANTS="a b" [ROUNDS=2] tools/mlp_variants.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in $(seq ${ROUNDS:-2}); do
  for v in product ${VARIANTS:?}; do
    if [ $v = product ]; then unset DGS_LIB; else export DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_$v.so; fi
    timeout -k 10 200 python tools/mlp_time.py --iters ${ITERS:-10} > gpurun_out/mlpv.log 2>&1 || { tail -5 gpurun_out/mlpv.log; exit 1; }
    tail -1 gpurun_out/mlpv.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())['split']; print('$v', {k: round(v, 4) for k, v in d.items()})"
  done
done

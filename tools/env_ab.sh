#!/bin/bash
# Alternating bench runs: product defaults vs the same library with an environment switch.
#   ENVAB="DGS_BLEND1=1" [RUNS=3] [TIMING=major] tools/env_ab.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in $(seq ${RUNS:-3}); do
  for v in default switched; do
    if [ $v = default ]; then E=""; else E="${ENVAB:?}"; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-timing ${TIMING:-major} ${BENCH_ARGS:-} > gpurun_out/envab.log 2>&1 || { tail -5 gpurun_out/envab.log; exit 1; }
    tail -1 gpurun_out/envab.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());k=d['kernels_ms_per_step']
print('$v', round(d['value'],1), round(d['ms_per_step'],3), {a: round(b,4) for a,b in k.items()})"
  done
done

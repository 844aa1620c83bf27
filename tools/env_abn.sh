#!/bin/bash
# Alternating bench runs over several environment variants (';'-separated; "default" = none):
#   ENVS="default;DGS_MLP_BWD8=1;DGS_MLP_FWD8=0" [RUNS=3] [TIMING=all] tools/env_abn.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
IFS=';' read -ra VS <<< "${ENVS:?}"
for i in $(seq ${RUNS:-3}); do
  for v in "${VS[@]}"; do
    E=""; [ "$v" != default ] && E="$v"
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-timing ${TIMING:-all} ${BENCH_ARGS:-} > gpurun_out/envab.log 2>&1 || { tail -5 gpurun_out/envab.log; exit 1; }
    tail -1 gpurun_out/envab.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());k=d['kernels_ms_per_step']
print('$v', round(d['value'],1), round(d['ms_per_step'],3), {a: round(b,4) for a,b in k.items() if b > 0.012})"
  done
done

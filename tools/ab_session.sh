#!/bin/bash
# Alternating default-flag bench runs: product library vs lib/diag/libdgs_base.so (tools/ab_build.sh)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in $(seq ${RUNS:-3}); do
  for v in product base; do
    if [ $v = base ]; then export DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_base.so; else unset DGS_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    tail -1 gpurun_out/ab.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v', round(d['value'],1), round(d['ms_per_step'],3))"
  done
done

#!/bin/bash
# Raster variant timing: bench.py with every kernel class timed, for the product library and for
# each lib/diag/libdgs_<name>.so in $DIAGS; prints kernels_ms_per_step and iters/s per run.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {
  timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --kernel-timing all > gpurun_out/rs.log 2>&1
  rc=$?
  echo "$1 rc=$rc $(python3 -c "import json;d=json.loads(open('gpurun_out/rs.log').read().strip().splitlines()[-1]);print(round(d['value'],1), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})")"
  return $rc
}
run product || exit 1
for v in ${DIAGS:-}; do
  DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_$v.so run $v || exit 1
done

#!/bin/bash
# MLP GPU tests (k_tgrad / k_dw_reduce changes), then two bench lines with every class timed
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/small_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/small_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/mlp_time.py --iters 10 > gpurun_out/small_mlpt.log 2>&1 || exit 1
tail -1 gpurun_out/small_mlpt.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/small_b$i.log 2>&1 || exit 1
  tail -1 gpurun_out/small_b$i.log | cut -c1-150
done
if [ -f deformable-3d-gaussians_amd/lib/diag/libdgs_base.so ]; then  # A/B vs raster.hip of HEAD
  for i in 1 2; do
    for L in base new; do
      if [ $L = base ]; then export DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_base.so; else unset DGS_LIB; fi
      timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-timing major > gpurun_out/ab_$L.log 2>&1 || exit 1
      tail -1 gpurun_out/ab_$L.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$L', round(d['value'],1), {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items() if k.startswith('blend')})"
    done
  done
fi

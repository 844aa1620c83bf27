#!/bin/bash
# raster GPU tests, then A/B of the preprocess kernels (HEAD raster.hip in lib/diag/libdgs_base.so)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_render.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pre_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pre_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for L in base new; do
    if [ $L = base ]; then export DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_base.so; else unset DGS_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-timing all > gpurun_out/pre_$L.log 2>&1 || exit 1
    tail -1 gpurun_out/pre_$L.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$L', round(d['value'],1), {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items() if k.startswith(('pre','blend'))})"
  done
done

#!/bin/bash
# raster + render GPU test files in one process (the order that failed once), current raster.hip and HEAD's
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_render.py -q --timeout 120 --timeout-method thread > gpurun_out/pc_new_$i.log 2>&1
  echo "new $i rc=$?"; tail -1 gpurun_out/pc_new_$i.log; grep FAILED gpurun_out/pc_new_$i.log
  DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_base.so timeout -k 10 300 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_render.py -q --timeout 120 --timeout-method thread > gpurun_out/pc_base_$i.log 2>&1
  echo "base $i rc=$?"; tail -1 gpurun_out/pc_base_$i.log; grep FAILED gpurun_out/pc_base_$i.log
done
exit 0

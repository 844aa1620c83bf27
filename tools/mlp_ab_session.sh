#!/bin/bash
# MLP change: MLP GPU tests, MLP timings new vs HEAD's mlp_split.hip (lib/diag/libdgs_base.so), phase profile
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mlpab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/mlpab_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_base.so timeout -k 10 200 python tools/mlp_time.py --iters 20 > gpurun_out/mlpab_base.log 2>&1 || exit 1
  echo base $(tail -1 gpurun_out/mlpab_base.log | cut -c1-120)
  timeout -k 10 200 python tools/mlp_time.py --iters 20 > gpurun_out/mlpab_new.log 2>&1 || exit 1
  echo new $(tail -1 gpurun_out/mlpab_new.log | cut -c1-120)
done
DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_prof.so timeout -k 10 200 python tools/mlp_phase.py 2>&1 | grep -v amdgpu.ids | head -24

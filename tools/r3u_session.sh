#!/bin/bash
# Round-3 A/B session: (1) raster / render / step-parity GPU tests on the product library,
# (2) MLP tests under lib/diag/libdgs_gate.so (k_dws barrier-free variant), (3) MLP kernel times
# product vs gate, (4) bench A/B product vs lib/diag/libdgs_base.so (tools/ab_build.sh).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_render.py tests/test_gpu_step_parity.py \
  -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/u_raster_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/u_raster_tests.txt; [ $rc -eq 0 ] || exit $rc
DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_gate.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py \
  -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/u_gate_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/u_gate_tests.txt; [ $rc -eq 0 ] || exit $rc
VARIANTS=gate ROUNDS=3 bash tools/mlp_variants.sh || exit $?
VARIANT=base TESTS="" RUNS=3 bash tools/variant_session.sh

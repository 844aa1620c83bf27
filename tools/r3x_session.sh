#!/bin/bash
# MLP GPU tests on the product (k_fwd xyz loaded once, k_bwd dOut in one load, k_tgrad coalesced over
# 8 workgroups), MLP kernel times product vs lib/diag/libdgs_base.so (HEAD's mlp_split.hip), then
# bench A/B with every kernel class timed
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_step_parity.py tests/test_gpu_render.py \
  -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/x_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/x_tests.txt; [ $rc -eq 0 ] || exit $rc
VARIANTS=base ROUNDS=3 bash tools/mlp_variants.sh || exit $?
VARIANT=base TESTS="" RUNS=2 TIMING=major bash tools/variant_session.sh

#!/bin/bash
# Full GPU suite on the product, then bench A/B of the radix tile size (DGS_RADIX_ITEMS 8 / 16 vs
# the default 4 items per thread below 512k keys)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/v_gpu_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/v_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
ENVAB="DGS_RADIX_ITEMS=8" RUNS=2 TIMING=all bash tools/env_ab.sh || exit $?
ENVAB="DGS_RADIX_ITEMS=16" RUNS=2 TIMING=all bash tools/env_ab.sh

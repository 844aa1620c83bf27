#!/bin/bash
# radix sort tests (direct, vs numpy stable argsort) + raster tests on the product, then a bench A/B
# against lib/diag/libdgs_base.so (HEAD's radix.hip: no copy-only pass), every kernel class timed
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_radix.py tests/test_gpu_raster.py -q -x --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/y_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/y_tests.txt; [ $rc -eq 0 ] || exit $rc
VARIANT=base TESTS="" RUNS=3 TIMING=all bash tools/variant_session.sh

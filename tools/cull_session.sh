#!/bin/bash
# raster + render GPU tests (tile-culled blend), then bench lines with the blend kernels timed
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cull_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/cull_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-timing major > gpurun_out/cull_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/cull_$i.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['value'],1), {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items()})"
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/cull_default.log 2>&1 || exit 1
tail -1 gpurun_out/cull_default.log | cut -c1-200

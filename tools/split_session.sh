#!/bin/bash
# GPU tests, then bench A/B: split-SH rasterizer (default) vs the concatenated SH rows
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/split_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    DGS_SPLIT_SH=$v timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-timing all > gpurun_out/split_$v.log 2>&1 || exit 1
    tail -1 gpurun_out/split_$v.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('split=$v', round(d['value'],1), {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items() if k.startswith(('pre','inp'))})"
  done
done

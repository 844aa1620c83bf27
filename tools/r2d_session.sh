#!/bin/bash
# bench lines (default, 6-DoF) with host timing, then the rocprofv3 trace + PMC passes (TAG=r2d)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for a in "" "--6dof" ""; do
  tag=$(echo "x$a" | tr -d ' -')
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > gpurun_out/r2d_bench_$tag.log 2>&1 || exit 1
  tail -1 gpurun_out/r2d_bench_$tag.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$a', round(d['value'],1), d['host_ms_per_step'])"
done
TAG=r2d PMC=${PMC:-1} bash tools/gpu_prof.sh

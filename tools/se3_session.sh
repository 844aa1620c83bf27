#!/bin/bash
# 6-DoF path: its GPU tests, then the bench with the fused screw (default) and with the torch glue (A/B)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_mlp.py -x -q --timeout 120 \
  --timeout-method thread -k "se3 or 6dof or fused" > gpurun_out/se3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/se3_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --6dof --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/se3_bench_fused_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/se3_bench_fused_$i.log | cut -c1-200
  DGS_SE3_GLUE=1 timeout -k 10 300 python bench.py --6dof --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/se3_bench_glue_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/se3_bench_glue_$i.log | cut -c1-200
done

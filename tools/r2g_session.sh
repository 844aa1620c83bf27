#!/bin/bash
# end-of-round evidence: smoke, every GPU test, default bench lines (first with cpu_baseline),
# 6-DoF line, then the rocprofv3 trace + PMC passes (TAG=r2g)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2g_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r2g_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2g_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r2g_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r2g_bench.jsonl
for a in "" "--no-cpu-baseline" "--no-cpu-baseline --6dof"; do
  timeout -k 10 300 python bench.py $a > gpurun_out/r2g_b.log 2>&1 || { tail -5 gpurun_out/r2g_b.log; exit 1; }
  tail -1 gpurun_out/r2g_b.log >> gpurun_out/r2g_bench.jsonl
  tail -1 gpurun_out/r2g_b.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$a', round(d['value'],1), round(d['roofline']['frac'],3), d['host_ms_per_step'])"
done
TAG=r2g bash tools/gpu_prof.sh

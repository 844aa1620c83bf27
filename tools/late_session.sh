#!/bin/bash
# GPU tests, then default bench lines (host timing) x3
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/late_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/late_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/late_b$i.log 2>&1 || { tail -5 gpurun_out/late_b$i.log; exit 1; }
  tail -1 gpurun_out/late_b$i.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['value'],1), d['host_ms_per_step'], d['config']['redone_steps'])"
done

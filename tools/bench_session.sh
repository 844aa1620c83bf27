#!/bin/bash
# Headline bench runs (default flags) N times, one JSON line each
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in $(seq ${RUNS:-2}); do
  timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$i.log 2>&1 || { tail -5 gpurun_out/bench_$i.log; exit 1; }
  tail -1 gpurun_out/bench_$i.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('bench', round(d['value'],1), 'iters/s', round(d['ms_per_step'],3), 'ms/step', d['roofline']['kernel'], round(d['roofline']['frac'],3), 'cpu', d['cpu_baseline'] and d['cpu_baseline'].get('value'))"
done

#!/bin/bash
# Alternating default-flag bench runs with and without an environment setting: ENVB="VAR=value"
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in $(seq ${RUNS:-3}); do
  for v in a b; do
    if [ $v = b ]; then E="$ENVB"; else E=""; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    tail -1 gpurun_out/ab.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v', round(d['value'],1), round(d['ms_per_step'],3), d['config'].get('redone_steps'))"
  done
done

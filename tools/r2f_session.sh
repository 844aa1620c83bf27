#!/bin/bash
# end-of-stage evidence: 3 default bench lines (with cpu_baseline on the first), then rocprofv3
# kernel trace + stats and the FETCH_SIZE / WRITE_SIZE passes (TAG=r2f)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/r2f_bench.jsonl
for a in "" "--no-cpu-baseline" "--no-cpu-baseline"; do
  timeout -k 10 300 python bench.py $a > gpurun_out/r2f_b.log 2>&1 || { tail -5 gpurun_out/r2f_b.log; exit 1; }
  tail -1 gpurun_out/r2f_b.log >> gpurun_out/r2f_bench.jsonl
  tail -1 gpurun_out/r2f_b.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['value'],1), d['roofline']['frac'], d['host_ms_per_step'])"
done
TAG=r2f bash tools/gpu_prof.sh

#!/bin/bash
# bench lines for the BASELINE.json configs that fit synthetic data (2: hellwarrior-sized 16k @400^2,
# 3: bouncingballs-sized 55k @800^2, 4: 6-DoF head), and the render FPS table (tools/fps.py)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r2e}
: > gpurun_out/${TAG}_configs.jsonl
for a in "--n 16000 --res 400" "--n 55000 --res 800" "--6dof" ""; do
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > gpurun_out/cfg.log 2>&1 || { tail -5 gpurun_out/cfg.log; exit 1; }
  tail -1 gpurun_out/cfg.log >> gpurun_out/${TAG}_configs.jsonl
  tail -1 gpurun_out/cfg.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$a', round(d['value'],1), d['config']['pairs_per_render'])"
done
timeout -k 10 300 python tools/fps.py > gpurun_out/${TAG}_render_fps.jsonl 2> gpurun_out/fps.err || { tail -5 gpurun_out/fps.err; exit 1; }
cat gpurun_out/${TAG}_render_fps.jsonl

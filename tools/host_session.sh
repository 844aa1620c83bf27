#!/bin/bash
# GPU tests (SSIM rewrite, Adam shared steps), bench lines, host cProfile of the step
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/host_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/host_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-timing all > gpurun_out/host_b$i.log 2>&1 || exit 1
  tail -1 gpurun_out/host_b$i.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['value'],1), d['host_ms_per_step'], {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items() if k.startswith(('ssim','blend','adam'))})"
done
timeout -k 10 300 python tools/host_cprofile.py > gpurun_out/host_cprofile.txt 2>&1 || exit 1
head -60 gpurun_out/host_cprofile.txt | tail -45

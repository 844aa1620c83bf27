#!/bin/bash
# GPU tests of the changed kernels, a bench line, then the dW L2-resident timing experiment
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r2e_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-timing all > gpurun_out/r2e_bench_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/r2e_bench_$i.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['value'],1), {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items()})"
done
bash tools/dw_l2_session.sh

#!/bin/bash
# One GPU session step by step: tests (optional $TESTS, pytest node ids / files), then bench runs of the
# product library and, with $AB=1, lib/diag/libdgs_base.so alternating ($RUNS rounds). Stops at the first
# fault / abort / timeout (rc >= 124 or a signal). Output: gpurun_out/$TAG/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-step}; mkdir -p gpurun_out/$T
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -v --timeout 300 --timeout-method thread -x > gpurun_out/$T/tests.txt 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/$T/tests.txt | tail -3
  if bad $rc; then exit $rc; fi
fi
for i in $(seq ${RUNS:-1}); do
  for v in product ${AB:+base}; do
    if [ $v = product ]; then unset DGS_LIB; else export DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_base.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --kernel-timing ${KT:-all} ${BENCH_ARGS:-} > gpurun_out/$T/bench_${v}_$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "bench $v rc=$rc"; tail -5 gpurun_out/$T/bench_${v}_$i.log; exit $rc; fi
    tail -1 gpurun_out/$T/bench_${v}_$i.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());k=d['kernels_ms_per_step']
print('$v', round(d['value'],1), {a: round(b,4) for a,b in k.items() if b > 0.015})"
  done
done
exit 0

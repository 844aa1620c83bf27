#!/bin/bash
# A/B of a diagnostic library variant (tools/build_diag.sh) against the product library on the GPU
# box: the raster parity tests under the variant, then alternating bench runs with per-kernel-class
# HIP-event timing.  usage: VARIANT=quad [TESTS="tests/test_gpu_raster.py"] [RUNS=3] tools/variant_session.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
V=${VARIANT:?}
LIBV=deformable-3d-gaussians_amd/lib/diag/libdgs_$V.so
if [ -n "${TESTS-tests/test_gpu_raster.py}" ]; then
  DGS_LIB=$LIBV timeout -k 10 300 python -m pytest ${TESTS-tests/test_gpu_raster.py} -q -x --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/variant_${V}_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/variant_${V}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq ${RUNS:-3}); do
  for v in product $V; do
    if [ $v = product ]; then unset DGS_LIB; else export DGS_LIB=$LIBV; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-timing ${TIMING:-major} ${BENCH_ARGS:-} > gpurun_out/variant.log 2>&1 || { tail -5 gpurun_out/variant.log; exit 1; }
    tail -1 gpurun_out/variant.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());k=d['kernels_ms_per_step']
print('$v', round(d['value'],1), round(d['ms_per_step'],3), {a: round(b,4) for a,b in k.items()})"
  done
done

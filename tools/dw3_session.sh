#!/bin/bash
# dW variant session: MLP GPU tests under DGS_MLP_SPLIT_DW=$MODE, then alternating timings of mode 0 / $MODE
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MODE=${MODE:-3}
if [ "${TESTS:-1}" = "1" ]; then
  DGS_MLP_SPLIT_DW=$MODE timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dw_test.log 2>&1
  rc=$?; echo "test rc=$rc"; tail -3 gpurun_out/dw_test.log
  [ $rc -eq 0 ] || exit $rc
fi
for m in 0 $MODE 0 $MODE; do
  DGS_MLP_SPLIT_DW=$m timeout -k 10 120 python tools/mlp_time.py --iters 20 > gpurun_out/dw_time.log 2>&1
  rc=$?; echo "mode $m rc=$rc $(python3 tools/dw_timefmt.py gpurun_out/dw_time.log)"
  [ $rc -eq 0 ] || exit $rc
done
for v in ${DIAGS:-}; do
  DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_$v.so DGS_MLP_SPLIT_DW=$MODE timeout -k 10 120 python tools/mlp_time.py --iters 20 > gpurun_out/dw_time.log 2>&1
  rc=$?; echo "diag $v rc=$rc $(python3 tools/dw_timefmt.py gpurun_out/dw_time.log)"
  [ $rc -eq 0 ] || exit $rc
done

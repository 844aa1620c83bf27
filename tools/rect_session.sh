#!/bin/bash
# rect binning vs sort binning: raster/render GPU tests, bitwise render comparison of the bench
# scene, step timings of both (every kernel class timed)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_render.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rect_test.log 2>&1
rc=$?; echo "test rc=$rc"; tail -3 gpurun_out/rect_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/sort_check.py gpurun_out/bin_rect.npz > gpurun_out/sc1.log 2>&1 || { echo "check rect failed"; tail -5 gpurun_out/sc1.log; exit 1; }
DGS_BINNING=sort timeout -k 10 200 python tools/sort_check.py gpurun_out/bin_sort.npz > gpurun_out/sc2.log 2>&1 || { echo "check sort failed"; exit 1; }
python3 -c "
import numpy as np
a=np.load('gpurun_out/bin_rect.npz'); b=np.load('gpurun_out/bin_sort.npz')
for k in a.files:
    d=np.abs(a[k].astype(np.float64)-b[k]).max(); print(k, 'bitwise' if np.array_equal(a[k],b[k]) else 'maxdiff %.3g (ref max %.3g)'%(d, np.abs(b[k]).max()))
"
bash tools/raster_session.sh || exit 1
DGS_BINNING=sort bash tools/raster_session.sh | sed "s/^product/sort/"

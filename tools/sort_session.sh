#!/bin/bash
# radix.hip vs hipcub binning: raster/render GPU tests, bitwise render comparison, step timings
# (default radix tiles, DGS_RADIX_ITEMS=4/8/16, hipcub)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_render.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sort_test.log 2>&1
rc=$?; echo "test rc=$rc"; tail -3 gpurun_out/sort_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/sort_check.py gpurun_out/sort_new.npz > gpurun_out/sc1.log 2>&1 || { echo "check new failed"; tail -5 gpurun_out/sc1.log; exit 1; }
DGS_HIPCUB_SORT=1 timeout -k 10 200 python tools/sort_check.py gpurun_out/sort_cub.npz > gpurun_out/sc2.log 2>&1 || { echo "check cub failed"; exit 1; }
python3 -c "
import numpy as np
a=np.load('gpurun_out/sort_new.npz'); b=np.load('gpurun_out/sort_cub.npz')
for k in a.files:
    d=np.abs(a[k].astype(np.float64)-b[k]).max(); print(k, 'bitwise' if np.array_equal(a[k],b[k]) else 'maxdiff %.3g (ref max %.3g)'%(d, np.abs(b[k]).max()))
"
for it in 4 16; do DGS_RADIX_ITEMS=$it bash tools/raster_session.sh | sed "s/^product/items$it/" || exit 1; done
bash tools/raster_session.sh || exit 1
DGS_HIPCUB_SORT=1 bash tools/raster_session.sh | sed "s/^product/hipcub/"

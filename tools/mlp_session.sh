#!/bin/bash
# MLP iteration: split-MLP GPU tests, per-phase cycle stamps (DGS_MLP_PROFILE diag build), bench
# with every kernel class timed
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mlp_test.log 2>&1
rc=$?; echo "test rc=$rc"; tail -3 gpurun_out/mlp_test.log
[ $rc -eq 0 ] || exit $rc
if [ -f deformable-3d-gaussians_amd/lib/diag/libdgs_prof.so ]; then
  DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_prof.so timeout -k 10 200 python tools/mlp_phase.py || exit 1
fi
bash tools/raster_session.sh
if [ "${TAILCHECK:-0}" = "1" ]; then
  timeout -k 10 200 python tools/tail_check.py gpurun_out/tail_on.npz || exit 1
  DGS_MLP_NO_TAIL=1 timeout -k 10 200 python tools/tail_check.py gpurun_out/tail_off.npz || exit 1
  python3 -c "
import numpy as np
a=np.load('gpurun_out/tail_on.npz'); b=np.load('gpurun_out/tail_off.npz')
bad=[k for k in a.files if not np.array_equal(a[k], b[k])]
print('tail split vs 64-point blocks:', 'bitwise identical' if not bad else 'DIFFER in %s' % bad[:8], '(%d arrays)' % len(a.files))
"
  DGS_MLP_NO_TAIL=1 bash tools/raster_session.sh | sed "s/^product/notail/"
fi

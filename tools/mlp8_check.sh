#!/bin/bash
# the 8-wave MLP kernels (k_fwd8 / k_bwd8: VAR=DGS_MLP_FWD8 | DGS_MLP_BWD8) vs the 16-wave ones: bitwise MLP outputs / gradients (tools/lib_bitwise.py),
# the MLP GPU tests, then the alternating bench A/B (tools/env_ab.sh). Output: gpurun_out/$TAG/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-fwd8}; mkdir -p gpurun_out/$T
env ${VAR:-DGS_MLP_FWD8}=${OFF:-0} timeout -k 10 300 python tools/lib_bitwise.py dump gpurun_out/$T/w16.npz || exit 1
timeout -k 10 300 python tools/lib_bitwise.py dump gpurun_out/$T/w8.npz || exit 1
python tools/lib_bitwise.py cmp gpurun_out/$T/w16.npz gpurun_out/$T/w8.npz | tee gpurun_out/$T/bitwise.txt
rm -f gpurun_out/$T/*.npz
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_native_step.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.txt 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.txt; [ $rc -ge 124 ] && exit $rc
ENVAB="${VAR:-DGS_MLP_FWD8}=${OFF:-0}" RUNS=${RUNS:-3} TIMING=all bash tools/env_ab.sh | tee gpurun_out/$T/ab.txt

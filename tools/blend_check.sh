#!/bin/bash
# Renders + gradients of the bench scene with the product library and lib/diag/libdgs_base.so
# (tools/ab_build.sh), compared: images / radii must be bitwise equal
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 200 python tools/sort_check.py gpurun_out/bc_new.npz > gpurun_out/bc1.log 2>&1 || { tail -5 gpurun_out/bc1.log; exit 1; }
DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_base.so timeout -k 10 200 python tools/sort_check.py gpurun_out/bc_base.npz > gpurun_out/bc2.log 2>&1 || { tail -5 gpurun_out/bc2.log; exit 1; }
python3 -c "
import numpy as np
a=np.load('gpurun_out/bc_new.npz'); b=np.load('gpurun_out/bc_base.npz')
for k in a.files:
    d=np.abs(a[k].astype(np.float64)-b[k]).max(); print(k, 'bitwise' if np.array_equal(a[k],b[k]) else 'maxdiff %.3g (ref max %.3g)'%(d, np.abs(b[k]).max()))
"

#!/bin/bash
# Baseline library for A/B timing: source file $SRC (default raster) taken from git revision $REV
# (default HEAD) and linked with the other current product objects -> lib/diag/libdgs_base.so
set -eu
cd "$(dirname "$0")/.."
SRC=${SRC:-raster}; REV=${REV:-HEAD}
git show $REV:deformable-3d-gaussians_amd/csrc/$SRC.hip > deformable-3d-gaussians_amd/csrc/${SRC}_abbase.hip
EXCL=$SRC SRC=${SRC}_abbase bash tools/build_diag.sh base= || true
rm -f deformable-3d-gaussians_amd/csrc/${SRC}_abbase.hip

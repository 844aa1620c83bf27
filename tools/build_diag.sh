#!/bin/bash
# Diagnostic variants of libdgs_hip.so (timing experiments, wrong results): one source file ($SRC,
# default mlp_split) rebuilt with <flags> (e.g. -DFOO) and linked with the other product objects into
# lib/diag/libdgs_<name>.so; use with DGS_LIB=...   usage: [SRC=raster] build_diag.sh name=flags ...
set -eu
cd "$(dirname "$0")/../deformable-3d-gaussians_amd"
SRC=${SRC:-mlp_split}
make -s -C csrc
mkdir -p lib/diag build_obj/diag
for v in "$@"; do
  name=${v%%=*}; flags=${v#*=}
  extra=""; [[ $SRC == mlp_split* ]] && extra="-mllvm -amdgpu-atomic-optimizer-strategy=None"  # as csrc/Makefile
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $extra $flags -c csrc/$SRC.hip -o build_obj/diag/${SRC}_$name.o
  objs=$(ls build_obj/*.o | grep -v "/${EXCL:-$SRC}.o")
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/diag/libdgs_$name.so $objs build_obj/diag/${SRC}_$name.o
  echo "built lib/diag/libdgs_$name.so ($SRC.hip $flags)"
done

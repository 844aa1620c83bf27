#!/bin/bash
# Diagnostic variants of libdgs_hip.so (timing experiments, wrong results): mlp_split.hip rebuilt with
# <flags> (e.g. -DFOO -fno-slp-vectorize) and linked with the product objects into lib/diag/libdgs_<name>.so; use with DGS_LIB=...
set -eu
cd "$(dirname "$0")/../deformable-3d-gaussians_amd"
make -s -C csrc
mkdir -p lib/diag build_obj/diag
for v in "$@"; do
  name=${v%%=*}; flags=${v#*=}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $flags -c csrc/mlp_split.hip -o build_obj/diag/mlp_split_$name.o
  objs=$(ls build_obj/*.o | grep -v mlp_split.o)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/diag/libdgs_$name.so $objs build_obj/diag/mlp_split_$name.o
  echo "built lib/diag/libdgs_$name.so ($flags)"
done

set -u
for v in prof noepi astatic; do
  echo "== $v"
  DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_$v.so timeout -k 10 200 python tools/mlp_phase.py 2>&1 | grep -E "mean block|L3 |slowest|L1 gemm|L1 epi" || exit 1
done

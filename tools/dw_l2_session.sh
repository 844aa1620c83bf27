set -u
cd /root/repo
timeout -k 10 200 python3 tools/mlp_time.py --iters 10 > gpurun_out/mlpt_base.log 2>&1 || exit 1
tail -3 gpurun_out/mlpt_base.log
DGS_LIB=deformable-3d-gaussians_amd/lib/diag/libdgs_dwsl2.so timeout -k 10 200 python3 tools/mlp_time.py --iters 10 > gpurun_out/mlpt_l2.log 2>&1 || exit 1
tail -3 gpurun_out/mlpt_l2.log

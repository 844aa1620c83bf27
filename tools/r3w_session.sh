#!/bin/bash
# MLP + loss GPU tests on the product (k_tgrad over 8 workgroups, unrolled SSIM tile loads), then a
# bench A/B against lib/diag/libdgs_base.so (HEAD's ssim.hip) with every kernel class timed, then a
# rocprofv3 kernel-stats pass of the product bench (k_tgrad)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_loss.py tests/test_gpu_step_parity.py \
  -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/w_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/w_tests.txt; [ $rc -eq 0 ] || exit $rc
VARIANT=base TESTS="" RUNS=2 TIMING=all bash tools/variant_session.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_w -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/w_bench_trace.log 2>&1 || exit $?
f=$(find gpurun_out/prof_w -name "*kernel_trace.csv" | head -1)
python3 tools/trace_gaps.py $f > gpurun_out/prof_w/trace_summary.txt 2>&1
head -30 gpurun_out/prof_w/trace_summary.txt

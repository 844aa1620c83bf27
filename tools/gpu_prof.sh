#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (summaries copied to profiles/ afterwards).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-r1}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_$TAG/bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 gpurun_out/prof_$TAG/bench.log
find gpurun_out/prof_$TAG -name "*stats*" | head
exit $rc

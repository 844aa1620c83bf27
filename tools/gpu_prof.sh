#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in
# passes of their own (no tracing alongside --pmc). Summaries are copied to profiles/ afterwards.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 $OUT/bench_trace.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
if [ "${PMC:-1}" = "1" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- \
      python3 bench.py --steps ${PMC_STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench_$C.log 2>&1
    rc=$?; echo "pmc $C rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
fi
find $OUT -name "*.csv" | head -20
exit 0

#!/bin/bash
# Round-3 evidence session: full GPU suite, smoke, default bench, rocprofv3 trace + PMC traffic
# passes (tools/gpu_prof.sh), each step under its own time limit; stops at the first failure.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-r3}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.jsonl 2> gpurun_out/${T}_bench.err || exit $?
tail -1 gpurun_out/${T}_bench.jsonl | cut -c1-200
TAG=$T STEPS=20 WARMUP=5 bash tools/gpu_prof.sh > gpurun_out/${T}_prof.log 2>&1 || { tail -5 gpurun_out/${T}_prof.log; exit 1; }
f=$(find gpurun_out/prof_$T/trace -name "*kernel_trace.csv" | head -1)
python3 tools/trace_gaps.py $f > gpurun_out/prof_$T/trace_summary.txt 2>&1
head -12 gpurun_out/prof_$T/trace_summary.txt

#!/bin/bash
# One GPU session: optional test files ($TESTS, names under tests/ without .py), then the alternating
# A/B of tools/ab_libs.sh over $VARIANTS ($RUNS rounds). Output: gpurun_out/$TAG/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-ab}; mkdir -p gpurun_out/$T
if [ -n "${TESTS:-}" ]; then
  files=$(echo "$TESTS" | tr ',' '\n' | sed 's|^|tests/|; s|$|.py|' | tr '\n' ' ')
  timeout -k 10 600 python -u -m pytest $files -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$T/tests.txt 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$T/tests.txt
  [ $rc -ge 124 ] && exit $rc
fi
bash tools/ab_libs.sh 2>&1 | tee gpurun_out/$T/ab.txt

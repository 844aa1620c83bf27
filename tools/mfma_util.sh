#!/bin/bash
# one rocprofv3 --pmc pass (no tracing) of the MFMA busy cycles and GUI-active cycles over a short bench
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/mfma_${TAG:-r2g}
mkdir -p $OUT
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?; echo "mfma pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/mfma_util.py $OUT

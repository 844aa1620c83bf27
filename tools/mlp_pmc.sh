#!/bin/bash
# Counter passes over the MLP-only driver (one rocprofv3 --pmc pass per counter group, no tracing).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/mlp_pmc_${TAG:-a}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $GROUP --output-format csv -d $OUT/p$i -o run -- \
    python3 tools/mlp_only.py --iters 3 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($GROUP) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done <<EOF
${PMC_GROUPS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS}
EOF
exit 0

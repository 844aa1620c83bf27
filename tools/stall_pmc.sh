#!/bin/bash
# Wave-state PMC passes (no tracing alongside --pmc) over tools/mlp_time.py (or PROG, a python script +
# args, e.g. PROG="bench.py --steps 6 --warmup 3 --no-cpu-baseline"): where the kernels' wave cycles go
# (waiting on counters, waiting to issue, issuing VALU / LDS / VMEM / MFMA). KERNELS: see stall_summary.py
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/stall_${TAG:-r3}
mkdir -p $OUT
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL ${PMC_TIMEOUT:-90} rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o run -- \
    python3 ${PROG:-tools/mlp_time.py --iters 3} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 tools/stall_summary.py $OUT

#!/bin/bash
# One GPU session's evidence for profiles/: the GPU test suite, smoke(), the default bench line (with
# its CPU baseline), config-sized bench lines, and a rocprofv3 kernel trace + stats plus the FETCH_SIZE /
# WRITE_SIZE passes (tools/gpu_prof.sh). Every GPU step has its own time limit; a step that times out,
# aborts or faults ends the session (a failing test does not). Outputs: gpurun_out/$TAG/.
#   usage: TAG=r4b [PARTS="tests smoke bench configs prof ab stall tests:<file>,..."] tools/evidence.sh
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-r4}
O=gpurun_out/$TAG
mkdir -p $O
PARTS=${PARTS:-"tests smoke bench configs prof"}

run() {  # run <limit-s> <log> <cmd...>: stop the session on a timeout / abort / fault
  local lim=$1 log=$2
  shift 2
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  echo "[$(date +%T)] rc=$rc $*" | cut -c1-200
  if [ $rc -ge 124 ]; then echo "stopping: rc=$rc"; tail -20 "$log"; exit $rc; fi
  return $rc
}

for p in $PARTS; do
  case $p in
    tests)
      run 1100 $O/gpu_tests.txt python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
      tail -3 $O/gpu_tests.txt ;;
    tests:*)  # tests:<file>,<file>,... (names under tests/, without .py)
      files=$(echo "${p#tests:}" | tr ',' '\n' | sed 's|^|tests/|; s|$|.py|' | tr '\n' ' ')
      log=$O/tests_$(echo "${p#tests:}" | tr ',' '_' | cut -c1-60).txt
      run 1000 $log python -u -m pytest $files -v --timeout 600 --timeout-method thread
      tail -3 $log ;;
    ab)  # the segmented blend backward against the serial replay, kernel timings on
      for s in 0 1; do
        DGS_BLEND_SEG=$s run 200 $O/ab_seg$s.jsonl python bench.py --no-cpu-baseline --kernel-timing major
        tail -1 $O/ab_seg$s.jsonl | cut -c1-200
      done ;;
    smoke)
      run 300 $O/smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
      tail -1 $O/smoke.txt ;;
    bench)
      run 400 $O/bench.jsonl python bench.py
      tail -c 600 $O/bench.jsonl ;;
    configs)
      : > $O/configs.jsonl
      for a in "--n 16000 --res 400" "--n 55000 --res 800" "--6dof" "--n 78600 --res 800 --6dof"; do
        run 300 $O/cfg.log python bench.py --no-cpu-baseline $a && tail -1 $O/cfg.log >> $O/configs.jsonl
      done
      cut -c1-160 $O/configs.jsonl ;;
    stall)  # wave-state PMC of the blend kernels over a short bench run (both blend backward paths)
      for s in ${STALL_SEG:-0 1}; do
        DGS_BLEND_SEG=$s TAG=${TAG}_seg$s PROG="bench.py --steps 6 --warmup 3 --no-cpu-baseline" PMC_TIMEOUT=150 \
          KERNELS="blend_fwd=k_blend_fwd,blend_bwd2=k_blend_bwd2<,blend_bwd2s=k_blend_bwd2s" \
          run 400 $O/stall_seg$s.txt bash tools/stall_pmc.sh
        tail -30 $O/stall_seg$s.txt
      done ;;
    outlier)  # tests/diag/step_outlier.py on the composed-step case OUTLIER (default blender-cfg2)
      run 300 $O/outlier.txt python tests/diag/step_outlier.py ${OUTLIER:-blender-cfg2}
      tail -30 $O/outlier.txt ;;
    prof)
      TAG=$TAG run 1000 $O/prof.log bash tools/gpu_prof.sh
      tail -5 $O/prof.log ;;
  esac
done
exit 0

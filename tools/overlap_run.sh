set -u
# one GPU session: the composed-step parity file, then the collective-overlap probe (tools/overlap_probe.py):
# the A/B sweep and two rocprofv3 kernel traces (reserve 0 / 8) analysed for overlap
T=${TAG:-r5d}
cd /root/repo && mkdir -p gpurun_out/$T && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_step_parity.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.txt 2>&1
echo "tests rc=$?"; tail -4 gpurun_out/$T/gpu_tests.txt
timeout -k 10 300 python -u tools/overlap_probe.py --sweep > gpurun_out/$T/sweep.jsonl 2> gpurun_out/$T/sweep.err || { echo sweep failed; tail -5 gpurun_out/$T/sweep.err; exit 1; }
for k in 0 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/tr$k -o run -- python3 tools/overlap_probe.py --mode standin --reserve $k > gpurun_out/$T/tr$k.log 2>&1 || exit 1
  f=$(find gpurun_out/$T/tr$k -name "*kernel_trace.csv" | head -1)
  python3 tools/overlap_probe.py --analyze $f > gpurun_out/$T/tr$k.analysis.jsonl
done
cat gpurun_out/$T/sweep.jsonl; tail -1 gpurun_out/$T/tr0.analysis.jsonl; tail -1 gpurun_out/$T/tr8.analysis.jsonl

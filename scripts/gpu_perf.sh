# one gpurun call: GPU tests, a bench, and a rocprofv3 kernel-trace of a short bench (per-kernel
# durations: python scripts/trace_gaps.py gpurun_out/trace/run_kernel_trace.csv).  Each GPU step has
# its own time limit; any failure ends the script.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest ${TESTS:-tests} -x -q -m gpu -rf -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/trace.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/trace.log
exit $rc

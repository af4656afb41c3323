# one gpurun call: golden + parity tests, bench A/B of the host sync scheme, kernel trace.
# Each GPU step has its own time limit; any failure ends the script (no further GPU work).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_golden.py tests/test_gpu_parity.py -x -q -m gpu -rf -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
LH_EVENT_SYNC=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b_ev.log 2>&1; rc=$?
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b_new.log 2>&1; rc=$?
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/trace.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/trace.log
exit $rc

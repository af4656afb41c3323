# one gpurun call: GPU tests, smoke(), a short bench.  Each GPU step has its own
# time limit; a fault / abort / timeout ends the script (no further GPU work).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -rf -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/b.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b.log
exit $rc

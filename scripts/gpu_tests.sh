# one gpurun call: the named GPU test files (default: all), then a short bench unless NO_BENCH=1.
# Each GPU step has its own time limit; any failure ends the script (no further GPU work).
set -u
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 500 python -u -m pytest $TESTS -x -q -m gpu -rf -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
[ "${NO_BENCH:-0}" = "1" ] && exit 0
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b.log
exit $rc

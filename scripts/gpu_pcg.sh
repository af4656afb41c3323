# one gpurun call: PCG + golden + parity GPU tests, then a short bench.  Each GPU step has its
# own time limit; any failure ends the script (no further GPU work).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pcg.py tests/test_golden.py tests/test_gpu_parity.py -x -q -m gpu -rf \
    -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b.log
exit $rc

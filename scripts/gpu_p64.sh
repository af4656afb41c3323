# the global-memory solve tests and the bench with its side measurements (p64_window among them)
set -o pipefail
mkdir -p gpurun_out/p64
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "ldlt or large_window or W32 or W24 or global or evaluate_only" > gpurun_out/p64/tests.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --steps 300 --warmup 3 --no-cpu > gpurun_out/p64/bench.json 2> gpurun_out/p64/bench.err

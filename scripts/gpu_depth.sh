# GPU tests, then solve throughput vs the number of trials kept enqueued ahead of the device
# (lh_options.trials_per_sync) and a kernel trace of the default
set -o pipefail
mkdir -p gpurun_out/depth
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/depth/tests.log 2>&1 || exit 1
fi
for d in 1 2 3; do
  timeout -k 10 120 python3 bench.py --steps 500 --warmup 3 --no-cpu --no-extras --trials-per-sync $d > gpurun_out/depth/d$d.json 2> gpurun_out/depth/d$d.err || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/depth/trn -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/depth/trn.log 2>&1

# the GPU suite, then two default-config bench lines without side measurements
set -u
mkdir -p gpurun_out/sb
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sb/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 120 python3 bench.py --steps 500 --warmup 3 --no-cpu --no-extras > gpurun_out/sb/b$r.json 2> gpurun_out/sb/b$r.err || exit 1
done

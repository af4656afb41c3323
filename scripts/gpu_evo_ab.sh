# GPU tests, then A/B of evaluate-only final-iteration trials (default) against full linearisation
# of every trial (LH_NO_EVO=1)
set -o pipefail
mkdir -p gpurun_out/evo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/evo/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 120 python3 bench.py --steps 500 --warmup 3 --no-cpu --no-extras > gpurun_out/evo/evo$r.json 2> gpurun_out/evo/evo$r.err || exit 1
  LH_NO_EVO=1 timeout -k 10 120 python3 bench.py --steps 500 --warmup 3 --no-cpu --no-extras > gpurun_out/evo/full$r.json 2> gpurun_out/evo/full$r.err || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/evo/tr -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/evo/tr.log 2>&1

# the GPU suite, two default-config bench lines, then k_ctrl phase stamps on C3 (diagnostic build)
set -u
mkdir -p gpurun_out/sb
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sb/tests.log 2>&1 || { tail -30 gpurun_out/sb/tests.log; exit 1; }
tail -2 gpurun_out/sb/tests.log
for r in 1 2; do
  timeout -k 10 120 python3 bench.py --steps 500 --warmup 3 --no-cpu --no-extras > gpurun_out/sb/b$r.json 2> gpurun_out/sb/b$r.err || exit 1
done
LH_LIB=lego-slam_amd/lib/liblego_ba_stamps.so timeout -k 10 200 python scripts/ctrl_stamps.py C3 > gpurun_out/sb/ctrl_stamps_C3.log 2>&1 || exit 1
cat gpurun_out/sb/ctrl_stamps_C3.log

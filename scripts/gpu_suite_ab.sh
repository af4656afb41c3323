# the GPU suite, one default bench line, then an A/B of lib/liblego_ba_x.so against the default build
set -u
mkdir -p gpurun_out/sb
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sb/tests.log 2>&1 || exit 1
timeout -k 10 120 python3 bench.py --steps 500 --warmup 3 --no-cpu --no-extras > gpurun_out/sb/b1.json 2> gpurun_out/sb/b1.err || exit 1
LIB_A=lego-slam_amd/lib/liblego_ba.so LIB_B=lego-slam_amd/lib/liblego_ba_x.so STEPS=500 bash scripts/gpu_ab.sh

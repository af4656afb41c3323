# the GPU suite on the variant build lib/liblego_ba_x.so, then an A/B of it against the default build
set -u
mkdir -p gpurun_out/var
LH_LIB=lego-slam_amd/lib/liblego_ba_x.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/var/tests.log 2>&1 || exit 1
LIB_A=lego-slam_amd/lib/liblego_ba.so LIB_B=lego-slam_amd/lib/liblego_ba_x.so STEPS=${STEPS:-500} bash scripts/gpu_ab.sh

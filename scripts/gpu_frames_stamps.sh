set -u
mkdir -p gpurun_out
LH_LIB=lego-slam_amd/lib/liblego_ba_stamps.so timeout -k 10 200 python scripts/frames_stamps.py > gpurun_out/frames_stamps.log 2>&1 || exit 1

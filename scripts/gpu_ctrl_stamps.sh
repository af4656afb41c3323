set -u
mkdir -p gpurun_out
LH_LIB=lego-slam_amd/lib/liblego_ba_stamps.so timeout -k 10 200 python scripts/ctrl_stamps.py C3 > gpurun_out/ctrl_stamps.log 2>&1; echo "rc=$?" >> gpurun_out/ctrl_stamps.log

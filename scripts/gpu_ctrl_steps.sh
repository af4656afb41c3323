# k_ctrl phase stamps with the per-step split of the LDL^T loop (diagnostic build), C3
set -u
mkdir -p gpurun_out/cs
LH_LIB=lego-slam_amd/lib/liblego_ba_stamps.so timeout -k 10 200 python scripts/ctrl_stamps.py C3 > gpurun_out/cs/ctrl_stamps_C3.log 2>&1 || { cat gpurun_out/cs/ctrl_stamps_C3.log; exit 1; }
cat gpurun_out/cs/ctrl_stamps_C3.log

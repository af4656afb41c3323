# k_ctrl / k_ctrl_g phase stamps (diagnostic -DLH_STAMPS build) on C3 and a 64-keyframe window
set -u
mkdir -p gpurun_out
for c in C3 P64; do
  LH_LIB=lego-slam_amd/lib/liblego_ba_stamps.so timeout -k 10 200 python scripts/ctrl_stamps.py $c > gpurun_out/ctrl_stamps_$c.log 2>&1 || exit 1
done

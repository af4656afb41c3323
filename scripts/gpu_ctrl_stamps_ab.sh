#!/bin/bash
# k_ctrl phase stamps (diagnostic -DLH_STAMPS builds) of the current build and the variants in STAMP_LIBS
set -u
mkdir -p gpurun_out
: > gpurun_out/cstamps.log
for lib in lego-slam_amd/lib/liblego_ba_stamps.so ${STAMP_LIBS:-}; do
  echo "== $lib" >> gpurun_out/cstamps.log
  LH_LIB=$lib timeout -k 10 200 python scripts/ctrl_stamps.py C3 >> gpurun_out/cstamps.log 2>&1 || exit 1
done
cat gpurun_out/cstamps.log

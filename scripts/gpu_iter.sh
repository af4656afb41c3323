# Iteration check on the GPU: the full -m gpu suite, k_ctrl phase stamps, one bench line (no CPU leg).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -rf -x \
  > gpurun_out/t.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t.log
[ $rc -le 1 ] || exit $rc
LH_LIB=lego-slam_amd/lib/liblego_ba_stamps.so timeout -k 10 200 python scripts/ctrl_stamps.py C3 > gpurun_out/ctrl_stamps.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu --no-extras > gpurun_out/b.log 2>&1 || exit $?
exit $rc

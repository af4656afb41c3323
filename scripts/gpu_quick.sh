set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -rf -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b.log
timeout -k 5 120 lego-slam_amd/lib/ubench_ldlt 120 > gpurun_out/u.log 2>&1
timeout -k 5 120 lego-slam_amd/lib/ubench_ldlt_parts >> gpurun_out/u.log 2>&1
exit $rc

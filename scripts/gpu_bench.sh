# bench only (quick iteration)
set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/b.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b.log
exit $rc

mkdir -p gpurun_out
nproc > gpurun_out/host.txt; lscpu | head -20 >> gpurun_out/host.txt
timeout -k 10 900 python -m pytest tests -q -m gpu -rf -p no:cacheprovider > gpurun_out/t1.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t1.log
if [ $rc -le 1 ]; then timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/b1.log 2>&1; echo "rc=$?" >> gpurun_out/b1.log; fi

#!/bin/bash
# round 3: the GPU suite on the current tree, then the host-buffer lh_solve A/B (current vs LIB_OLD), twice
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r03b_tests.log 2>&1 || { tail -40 gpurun_out/r03b_tests.log; exit 1; }
tail -2 gpurun_out/r03b_tests.log
: > gpurun_out/r03b_host.txt
for r in 1 2; do
  timeout -k 10 120 python scripts/host_path_ab.py >> gpurun_out/r03b_host.txt 2>&1 || exit 1
  LH_LIB=$LIB_OLD timeout -k 10 120 python scripts/host_path_ab.py >> gpurun_out/r03b_host.txt 2>&1 || exit 1
done
cat gpurun_out/r03b_host.txt

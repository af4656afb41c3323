#!/bin/bash
# many-keyframe PCG (k_ctrl_p) tests first, then the whole GPU suite
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_pcg.py -x -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r03d_pcg.log 2>&1 || { tail -40 gpurun_out/r03d_pcg.log; exit 1; }
tail -3 gpurun_out/r03d_pcg.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r03d_tests.log 2>&1 || { tail -40 gpurun_out/r03d_tests.log; exit 1; }
tail -2 gpurun_out/r03d_tests.log

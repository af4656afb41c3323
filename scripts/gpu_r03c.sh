#!/bin/bash
# GPU suite, host-path detail (current vs LIB_OLD), and the timed line without side measurements
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r03c_tests.log 2>&1 || { tail -40 gpurun_out/r03c_tests.log; exit 1; }
tail -2 gpurun_out/r03c_tests.log
timeout -k 10 300 python scripts/host_path_detail.py > gpurun_out/r03c_host.txt 2>&1 || { cat gpurun_out/r03c_host.txt; exit 1; }
cat gpurun_out/r03c_host.txt
timeout -k 10 300 python bench.py --no-extras --no-cpu > gpurun_out/r03c_bench.json 2>/dev/null && python -c "
import json; d=json.load(open('gpurun_out/r03c_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernels_ms_per_solve_event_bracketed'])"

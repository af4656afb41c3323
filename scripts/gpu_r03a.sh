#!/bin/bash
# round 3, first GPU call: the whole GPU suite (incl. the C4 2/4-rank sharded parity tests), the
# C4 gate-0/gate-1 rank traces, then the default bench line.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r03a_tests.log 2>&1 && \
timeout -k 10 600 python -u scripts/c4_rank_traces.py > gpurun_out/r03a_traces.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err

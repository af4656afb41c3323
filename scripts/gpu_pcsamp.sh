#!/bin/bash
# PC sampling (stochastic, cycles) of k_lin replays: where its waves stall.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pcs
timeout -k 10 60 rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1 || { echo "rocprofv3 -L failed"; exit 1; }
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
    --pc-sampling-interval ${PCS_INTERVAL:-65536} -d gpurun_out/pcs/run -o pcs --output-format csv -- \
    python3 scripts/klin_replay.py 300 > gpurun_out/pcs/run.log 2>&1
rc=$?
echo "rc=$rc"; tail -5 gpurun_out/pcs/run.log; find gpurun_out/pcs/run -type f | head; du -sh gpurun_out/pcs
exit $rc

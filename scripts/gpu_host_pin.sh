#!/bin/bash
# Host-buffer path with the planner pool pinned to the caller's last-level cache (default) and not.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/host_path_detail.py > gpurun_out/host_pin1.txt 2>&1 || { tail -20 gpurun_out/host_pin1.txt; exit 1; }
LH_HOST_PIN=0 timeout -k 10 300 python3 -u scripts/host_path_detail.py > gpurun_out/host_pin0.txt 2>&1 || { tail -20 gpurun_out/host_pin0.txt; exit 1; }
echo "== pinned"; cat gpurun_out/host_pin1.txt; echo "== not pinned"; cat gpurun_out/host_pin0.txt

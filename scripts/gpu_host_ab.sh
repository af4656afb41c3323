#!/bin/bash
# Host-buffer path detail (planner stages, lh_solve parts; fresh vs reused output arrays) for the
# current build and LIB_OLD.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/host_path_detail.py > gpurun_out/host_ab.txt 2>&1 || { tail -20 gpurun_out/host_ab.txt; exit 1; }
cat gpurun_out/host_ab.txt

#!/bin/bash
# round 3 profiles: k_lin kernel trace of the timed bench (its replays + in-solve launches), the PMC passes
# (k_lin HBM traffic), a kernel-trace --stats summary of the whole bench with side lines, then the default
# bench line.  Each GPU step has its own limit; any failure ends the script.
set -u
mkdir -p gpurun_out/r03p
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/r03p/kl gpurun_out/r03p/st gpurun_out/pmc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03p/kl -o kl --output-format csv -- \
    python3 bench.py --steps 300 --warmup 3 --no-cpu --no-extras > gpurun_out/r03p/kl.log 2>&1 || exit 1
python3 scripts/rocprof_k_lin.py "$(find gpurun_out/r03p/kl -name '*kernel_trace.csv' | head -1)" \
    gpurun_out/r03p/r03_rocprof_k_lin.json C3-stable_noout-s0 || exit 1
cp "$(find gpurun_out/r03p/kl -name '*kernel_stats.csv' | head -1)" gpurun_out/r03p/r03_rocprof_kernel_stats_timed.csv
python3 scripts/rocprof_active.py "$(find gpurun_out/r03p/kl -name '*kernel_trace.csv' | head -1)" > gpurun_out/r03p/r03_rocprof_active_launches.txt 2>&1 || true
rm -rf gpurun_out/r03p/kl
bash scripts/gpu_pmc.sh || exit 1
python3 scripts/pmc_traffic.py gpurun_out/pmc gpurun_out/r03p/r03_pmc_k_lin.json C3-stable_noout-s0 || exit 1
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/r03p/r03_pmc_summary.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03p/st -o st --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/r03p/st.log 2>&1 || exit 1
cp "$(find gpurun_out/r03p/st -name '*kernel_stats.csv' | head -1)" gpurun_out/r03p/r03_rocprof_kernel_stats_all.csv
rm -rf gpurun_out/r03p/st gpurun_out/pmc/*/
# the bench line reads the committed trace / PMC files: use this run's
cp gpurun_out/r03p/r03_rocprof_k_lin.json gpurun_out/r03p/r03_pmc_k_lin.json profiles/
timeout -k 10 400 python3 bench.py > gpurun_out/r03p/r03_bench.json 2> gpurun_out/r03p/r03_bench.err || exit 1
tail -c 3000 gpurun_out/r03p/r03_bench.json

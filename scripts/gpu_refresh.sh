# one gpurun call that refreshes everything under profiles/: the default bench line (with the CPU
# baseline), a rocprofv3 kernel-trace --stats summary of the same bench, and the PMC passes whose
# FETCH_SIZE/WRITE_SIZE give k_lin's HBM traffic.  Each GPU step has its own limit; any failure ends it.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/b_default.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b_default.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/prof.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc.sh

# L2 (TCC) hit/miss per kernel over the C3 bench: is k_ctrl's prologue load (the staged system written
# by k_reduce on every XCD, read by one CU) served from its XCD's L2 or from the fabric?
# Separate counter passes, each with --kernel-trace only.
set -u
mkdir -p gpurun_out/pmcl2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, counters...
    local nm=$1; shift
    timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmcl2/$nm -o $nm --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/pmcl2/$nm.log 2>&1
}
run tcc TCC_HIT_sum TCC_MISS_sum || exit $?
run tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmcl2 > gpurun_out/pmcl2/summary.txt
cat gpurun_out/pmcl2/summary.txt

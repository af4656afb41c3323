# the k_lin rocprofv3 trace of `bench.py --no-extras` (replays + in-solve launches -> profiles/r02_rocprof_k_lin.json),
# then the default bench line, which reports that file beside its live timing
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/profne
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profne -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras > gpurun_out/profne.log 2>&1 || exit 1
python3 scripts/rocprof_k_lin.py gpurun_out/profne/run_kernel_trace.csv profiles/r02_rocprof_k_lin.json C3-stable_noout-s0 || exit 1
cp profiles/r02_rocprof_k_lin.json gpurun_out/r02_rocprof_k_lin.json
timeout -k 10 400 python bench.py > gpurun_out/b_line.log 2>&1 || exit 1

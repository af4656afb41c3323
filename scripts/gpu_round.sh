# one gpurun call: tests, bench, stamps, rocprof kernel trace.  Each GPU step has its
# own time limit; a fault / abort / timeout ends the script (no further GPU work).
set -u
mkdir -p gpurun_out
ok() { [ "$1" -le 1 ]; }
timeout -k 10 900 python -m pytest tests -q -m gpu -rf -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t.log
ok $rc || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/b.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b.log
[ $rc -eq 0 ] || exit $rc
LH_LIB=lego-slam_amd/lib/liblego_ba_stamps.so timeout -k 10 300 python scripts/stamps.py C3 > gpurun_out/stamps.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/stamps.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/prof.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/prof.log
[ $rc -eq 0 ] || exit $rc

# round-2 closing refresh: full GPU suite (log kept), the default bench line with its CPU baseline,
# the rocprofv3 kernel-trace --stats summary, the PMC passes, and the frontend / LK kernel trace
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_refresh.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/lkprof -o lk --output-format csv -- \
  python3 scripts/frontend_lk_run.py > gpurun_out/lkprof.log 2>&1 || exit 1
python3 scripts/frontend_prof_summary.py "$(find gpurun_out/lkprof -name '*kernel_trace.csv' | head -1)" > gpurun_out/lk_summary.txt

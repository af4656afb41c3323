# k_frames kernel durations (rocprofv3 kernel trace of scripts/frontend_lk_run.py) for the default build (v0)
# and lib/liblego_ba_v1.so, alternating, plus the frontend tests on the variant
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fa
: > gpurun_out/fa/summary.txt
LH_LIB=lego-slam_amd/lib/liblego_ba_v1.so timeout -k 10 300 python -u -m pytest tests/test_frontend.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/fa/tests_v1.log 2>&1 || { tail -30 gpurun_out/fa/tests_v1.log; exit 1; }
tail -1 gpurun_out/fa/tests_v1.log
for r in 1 2; do
for v in 0 1; do
  lib=$( [ $v = 0 ] && echo lego-slam_amd/lib/liblego_ba.so || echo lego-slam_amd/lib/liblego_ba_v1.so )
  LH_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/fa/v$v.$r -o p --output-format csv -- \
    python3 scripts/frontend_lk_run.py > gpurun_out/fa/run_v$v.$r.log 2>&1 || exit 1
  echo "v$v.$r $(python3 scripts/frontend_prof_summary.py "$(find gpurun_out/fa/v$v.$r -name '*kernel_trace.csv' | head -1)" | grep k_frames)" >> gpurun_out/fa/summary.txt
  rm -rf gpurun_out/fa/v$v.$r
done
done
cat gpurun_out/fa/summary.txt

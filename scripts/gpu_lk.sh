# one gpurun call: the LK GPU tests and a rocprofv3 kernel trace of the frontend paths
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lk.py -m gpu \
  > gpurun_out/lk_tests.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/lkprof -o lk --output-format csv -- \
  python3 scripts/frontend_lk_run.py > gpurun_out/lkprof.log 2>&1 || exit 1
python3 scripts/frontend_prof_summary.py "$(find gpurun_out/lkprof -name '*kernel_trace.csv' | head -1)" \
  > gpurun_out/lk_summary.txt

# one gpurun call: the frontend GPU tests, the k_frames phase stamps, and a rocprofv3 kernel trace of the frontend paths
set -o pipefail
mkdir -p gpurun_out/fe
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_frontend.py tests/test_lk.py -m gpu \
  > gpurun_out/fe/tests.log 2>&1 || exit 1
LH_LIB=lego-slam_amd/lib/liblego_ba_stamps.so timeout -k 10 200 python scripts/frames_stamps.py > gpurun_out/fe/stamps.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/fe/prof -o fe --output-format csv -- \
  python3 scripts/frontend_lk_run.py > gpurun_out/fe/prof.log 2>&1 || exit 1
python3 scripts/frontend_prof_summary.py "$(find gpurun_out/fe/prof -name '*kernel_trace.csv' | head -1)" \
  > gpurun_out/fe/summary.txt

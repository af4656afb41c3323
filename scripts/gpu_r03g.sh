# the GPU suite on the current build, then the N-way rocprof A/B against VARIANTS
set -u
mkdir -p gpurun_out/sb
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/sb/tests.log 2>&1 || { tail -40 gpurun_out/sb/tests.log; exit 1; }
tail -1 gpurun_out/sb/tests.log
bash scripts/gpu_abn.sh

# final evidence on the final tree: the GPU suite, smoke(), the default bench line
set -u
mkdir -p gpurun_out/fin
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/fin/r03_gpu_tests_final.log 2>&1 || { tail -40 gpurun_out/fin/r03_gpu_tests_final.log; exit 1; }
tail -1 gpurun_out/fin/r03_gpu_tests_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/r03_smoke_final.log 2>&1 || { cat gpurun_out/fin/r03_smoke_final.log; exit 1; }
cat gpurun_out/fin/r03_smoke_final.log
timeout -k 10 400 python3 bench.py > gpurun_out/fin/r03_bench_final.json 2> gpurun_out/fin/r03_bench_final.err || exit 1
tail -c 400 gpurun_out/fin/r03_bench_final.json

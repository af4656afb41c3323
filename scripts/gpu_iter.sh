# Iteration check on the GPU: the full -m gpu suite, one bench line (no CPU leg), and one PMC pass
# of the LDS counters over the bench.  Each GPU step has its own time limit; a failure ends it.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -rf -x \
  > gpurun_out/t.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu --no-extras > gpurun_out/b.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_lds
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES \
  -d gpurun_out/pmc_lds -o lds --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras \
  > gpurun_out/pmc_lds.log 2>&1 || exit $?
exit $rc

# Round-2 GPU call: GPU tests, the bench line, and a rocprofv3 kernel trace of the bench's timed path.
# Each GPU step has its own time limit; a failure, fault or timeout ends the script.
set -u
mkdir -p gpurun_out
STAGE=${1:-all}
if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
  timeout -k 10 1100 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -rf \
    > gpurun_out/t.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t.log
  [ $rc -le 1 ] || exit $rc
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/b.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$STAGE" = all ] || [ "$STAGE" = prof ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras > gpurun_out/prof.log 2>&1; rc=$?
  echo "rc=$rc" >> gpurun_out/prof.log
  [ $rc -eq 0 ] || exit $rc
fi
exit 0

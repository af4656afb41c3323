# the GPU suite on the current build, then rocprofv3 kernel traces of the C3 bench for the current
# build (A) and LIB_B alternating twice (per-kernel averages), then k_ctrl phase stamps on C3
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cab
: > gpurun_out/cab/summary.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/cab/tests.log 2>&1 || { tail -30 gpurun_out/cab/tests.log; exit 1; }
tail -1 gpurun_out/cab/tests.log
for r in 1 2; do
for v in A B; do
  lib=$( [ $v = A ] && echo lego-slam_amd/lib/liblego_ba.so || echo "$LIB_B" )
  LH_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/cab/$v.$r -o p --output-format csv -- \
    python3 bench.py --steps 300 --warmup 3 --no-cpu --no-extras > gpurun_out/cab/bench_$v.$r.log 2>&1 || exit 1
  for f in $(find gpurun_out/cab/$v.$r -name '*kernel_trace.csv'); do
    python3 scripts/rocprof_active.py "$f" | sed "s/^/$v.$r /" >> gpurun_out/cab/summary.txt
  done
  python3 -c "
import json,sys
for l in open('gpurun_out/cab/bench_$v.$r.log'):
    if l.startswith('{'): d=json.loads(l); print('$v.$r', 'ms_per_step', d['ms_per_step'], 'it/s', d['value'])" >> gpurun_out/cab/summary.txt
  rm -rf gpurun_out/cab/$v.$r
done
done
LH_LIB=lego-slam_amd/lib/liblego_ba_stamps.so timeout -k 10 200 python scripts/ctrl_stamps.py C3 > gpurun_out/cab/ctrl_stamps_C3.log 2>&1 || exit 1
cat gpurun_out/cab/summary.txt | grep -v 'k_frames\|k_lk\|k_gather\|k_reset\|k_nop'
cat gpurun_out/cab/ctrl_stamps_C3.log

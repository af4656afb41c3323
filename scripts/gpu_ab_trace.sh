#!/bin/bash
# Kernel A/B: the parity tests ($TESTS) on the current build, then rocprofv3 kernel traces of the C3
# bench (300 solves) for the current build (A) and LIB_B, alternating twice; per-kernel averages.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cab
TESTS=${TESTS:-tests/test_gpu_parity.py tests/test_golden.py tests/test_pcg.py}
: > gpurun_out/cab/summary.txt
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cab/tests.log 2>&1 || { tail -30 gpurun_out/cab/tests.log; exit 1; }
tail -1 gpurun_out/cab/tests.log
for r in 1 2; do
for v in A B; do
  lib=$( [ $v = A ] && echo lego-slam_amd/lib/liblego_ba.so || echo "$LIB_B" )
  LH_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/cab/$v.$r -o p --output-format csv -- \
    python3 bench.py --steps 300 --warmup 3 --no-cpu --no-extras > gpurun_out/cab/bench_$v.$r.log 2>&1 || exit 1
  for f in $(find gpurun_out/cab/$v.$r -name '*kernel_stats.csv'); do
    python3 - "$v.$r" "$f" >> gpurun_out/cab/summary.txt <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[2])):
    n = row.get("Name", "")
    if any(k in n for k in ("k_ctrl", "k_lin<3", "k_reduce")):
        print(sys.argv[1], n[:24], row.get("Calls"), row.get("AverageNs"))
PY
  done
  python3 -c "
import json,sys
for l in open('gpurun_out/cab/bench_$v.$r.log'):
    if l.startswith('{'): d=json.loads(l); print('$v.$r', 'ms_per_step', d['ms_per_step'], 'it/s', d['value'])" >> gpurun_out/cab/summary.txt
  rm -rf gpurun_out/cab/$v.$r
done
done
cat gpurun_out/cab/summary.txt

#!/bin/bash
# k_ctrl variants: k_ldlt probe parity on the current build, phase stamps of each stamps build in
# STAMP_LIBS, and rocprofv3 kernel-trace averages of the C3 bench (300 solves) for each product build in
# LIBS ("name=path ..."), two alternating rounds.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cv
: > gpurun_out/cv/summary.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "reduced_solve or single_trial or full_solve_parity_stable" \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cv/tests.log 2>&1 || { tail -30 gpurun_out/cv/tests.log; exit 1; }
tail -1 gpurun_out/cv/tests.log >> gpurun_out/cv/summary.txt
for lib in ${STAMP_LIBS:-}; do
  echo "== $lib" >> gpurun_out/cv/summary.txt
  LH_LIB=$lib timeout -k 10 200 python scripts/ctrl_stamps.py C3 >> gpurun_out/cv/summary.txt 2>&1 || exit 1
done
for r in 1 2; do
for nv in ${LIBS}; do
  v=${nv%%=*}; lib=${nv#*=}
  LH_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/cv/$v.$r -o p --output-format csv -- \
    python3 bench.py --steps 300 --warmup 3 --no-cpu --no-extras > gpurun_out/cv/bench_$v.$r.log 2>&1 || exit 1
  for f in $(find gpurun_out/cv/$v.$r -name '*kernel_stats.csv'); do
    python3 - "$v.$r" "$f" >> gpurun_out/cv/summary.txt <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[2])):
    n = row.get("Name", "")
    if any(k in n for k in ("k_ctrl", "k_lin<3, true>", "k_reduce")):
        print(sys.argv[1], n[:24], row.get("Calls"), row.get("AverageNs"))
PY
  done
  python3 -c "
import json
for l in open('gpurun_out/cv/bench_$v.$r.log'):
    if l.startswith('{'): d=json.loads(l); print('$v.$r', 'ms_per_step', d['ms_per_step'], 'it/s', d['value'])" >> gpurun_out/cv/summary.txt
  rm -rf gpurun_out/cv/$v.$r
done
done
cat gpurun_out/cv/summary.txt

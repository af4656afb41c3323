# k_ctrl / k_ldlt_probe kernel durations (rocprofv3 kernel trace) for the default build (v0) and the
# variant builds lib/liblego_ba_v<N>.so named in VARIANTS, two rounds, plus each variant's k_ctrl parity tests
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cm
: > gpurun_out/cm/summary.txt
for v in ${VARIANTS:-1}; do
  LH_LIB=lego-slam_amd/lib/liblego_ba_v$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/cm/tests_v$v.log 2>&1 || { echo "v$v tests failed"; tail -20 gpurun_out/cm/tests_v$v.log; exit 1; }
  tail -1 gpurun_out/cm/tests_v$v.log
done
for r in 1 2; do
for v in ${ORDER:-0 ${VARIANTS:-1}}; do
  lib=$( [ $v = 0 ] && echo lego-slam_amd/lib/liblego_ba.so || echo lego-slam_amd/lib/liblego_ba_v$v.so )
  LH_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/cm/v$v.$r -o p --output-format csv -- \
    python3 bench.py --steps 300 --warmup 3 --no-cpu --no-extras > gpurun_out/cm/bench_v$v.$r.log 2>&1 || exit 1
  for f in $(find gpurun_out/cm/v$v.$r -name '*kernel_stats.csv'); do
    python3 - "v$v.$r" "$f" >> gpurun_out/cm/summary.txt <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[2])):
    n = row.get("Name", "")
    if any(k in n for k in ("k_ctrl", "k_lin<3, true>", "k_lin<3, false>", "k_reduce")):
        print(sys.argv[1], n[:24], row.get("Calls"), row.get("AverageNs"))
PY
  done
  rm -rf gpurun_out/cm/v$v.$r
done
done
cat gpurun_out/cm/summary.txt

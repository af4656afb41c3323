# k_ctrl / k_ldlt_probe kernel durations under rocprofv3 for the default build (A) and lib/liblego_ba_x.so (B)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cab
for r in 1 2; do
for v in A B; do
  lib=$( [ $v = A ] && echo lego-slam_amd/lib/liblego_ba.so || echo lego-slam_amd/lib/liblego_ba_x.so )
  LH_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/cab/$v$r -o p --output-format csv -- \
    python3 bench.py --steps 300 --warmup 3 --no-cpu --no-extras > gpurun_out/cab/bench_$v$r.log 2>&1 || exit 1
  LH_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/cab/p$v$r -o p --output-format csv -- \
    python3 scripts/ldlt_probe_time.py > gpurun_out/cab/probe_$v$r.log 2>&1 || exit 1
  for f in $(find gpurun_out/cab/$v$r gpurun_out/cab/p$v$r -name '*kernel_stats.csv'); do
    python3 - "$v$r" "$f" >> gpurun_out/cab/summary.txt <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[2])):
    n = row.get("Name", "")
    if any(k in n for k in ("k_ctrl", "k_ldlt_probe", "k_lin", "k_reduce")):
        print(sys.argv[1], n[:40], row.get("Calls"), row.get("AverageNs"))
PY
  done
done
done
cat gpurun_out/cab/summary.txt
grep -h '^{' gpurun_out/cab/bench_*.log | python3 -c "import sys,json; [print(json.loads(l)['value']) for l in sys.stdin]"

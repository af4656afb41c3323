# k_ldlt_probe kernel duration (rocprofv3 kernel trace, 30 calls, n = 120) for the default build (v0) and lib/liblego_ba_v<N>.so
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pm
: > gpurun_out/pm/summary.txt
for r in 1 2; do
for v in 0 ${VARIANTS:-1}; do
  lib=$( [ $v = 0 ] && echo lego-slam_amd/lib/liblego_ba.so || echo lego-slam_amd/lib/liblego_ba_v$v.so )
  LH_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pm/v$v.$r -o p --output-format csv -- \
    python3 scripts/ldlt_probe_time.py > gpurun_out/pm/probe_v$v.$r.log 2>&1 || exit 1
  f=$(find gpurun_out/pm/v$v.$r -name '*kernel_stats.csv' | head -1)
  python3 - "v$v.$r" "$f" "$(grep residual gpurun_out/pm/probe_v$v.$r.log)" >> gpurun_out/pm/summary.txt <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[2])):
    if "k_ldlt_probe" in row.get("Name", ""):
        print(sys.argv[1], row.get("Calls"), row.get("AverageNs"), sys.argv[3])
PY
  rm -rf gpurun_out/pm/v$v.$r
done
done
cat gpurun_out/pm/summary.txt

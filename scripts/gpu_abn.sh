# N-way kernel A/B: golden parity on each variant library, then rocprofv3 kernel traces of the C3 bench
# (300 solves) for every variant in VARIANTS (lego-slam_amd/lib/liblego_ba_<v>.so; "A" = the default
# build), alternating twice; per-kernel averages over active launches.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abn
: > gpurun_out/abn/summary.txt
lib_of() { [ "$1" = A ] && echo lego-slam_amd/lib/liblego_ba.so || echo lego-slam_amd/lib/liblego_ba_$1.so; }
for v in $VARIANTS; do
  LH_LIB=$(lib_of $v) timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_golden.py} -m gpu -x -q --timeout 120 \
      --timeout-method thread -p no:cacheprovider > gpurun_out/abn/tests_$v.log 2>&1 || { tail -30 gpurun_out/abn/tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/abn/tests_$v.log)" >> gpurun_out/abn/summary.txt
done
for r in 1 2; do
for v in $VARIANTS; do
  LH_LIB=$(lib_of $v) timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/abn/$v.$r -o p --output-format csv -- \
    python3 bench.py --steps 300 --warmup 3 --no-cpu --no-extras > gpurun_out/abn/bench_$v.$r.log 2>&1 || exit 1
  for f in $(find gpurun_out/abn/$v.$r -name '*kernel_trace.csv'); do
    python3 scripts/rocprof_active.py "$f" | grep -E 'k_ctrl|k_lin<3, true|k_reduce' | sed "s/^/$v.$r /" >> gpurun_out/abn/summary.txt
  done
  python3 -c "
import json,sys
for l in open('gpurun_out/abn/bench_$v.$r.log'):
    if l.startswith('{'): d=json.loads(l); print('$v.$r', 'ms_per_step', d['ms_per_step'], 'it/s', d['value'])" >> gpurun_out/abn/summary.txt
  rm -rf gpurun_out/abn/$v.$r
done
done
cat gpurun_out/abn/summary.txt

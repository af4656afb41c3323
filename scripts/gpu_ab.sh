# A/B timing of two builds of liblego_ba.so in one box session (bench.py, no cpu leg), alternating.
#   LIB_A=... LIB_B=... bash scripts/gpu_ab.sh
set -u
mkdir -p gpurun_out
: > gpurun_out/ab.log
for r in 1 2; do
  for v in A B; do
    lib=$( [ $v = A ] && echo "$LIB_A" || echo "$LIB_B" )
    LH_LIB=$lib timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu ${AB_ARGS:---no-extras} > gpurun_out/ab_$v$r.log 2>&1 || exit $?
    python3 - "$v" gpurun_out/ab_$v$r.log >> gpurun_out/ab.log <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l)
        print(sys.argv[1], d['ms_per_step'], d['value'], d.get('roofline', {}).get('avg_launch_ms'))
PY
  done
done
cat gpurun_out/ab.log

# diagnostic: per-launch k_lin time (bench roofline.avg_launch_ms) for several builds, same box.
#   VARIANTS="A Vtasks ..." bash scripts/gpu_ab_lin.sh   (lego-slam_amd/lib/liblego_ba_<v>.so)
set -u
mkdir -p gpurun_out
: > gpurun_out/ab.log
for v in ${VARIANTS:-A B A B}; do
  LH_LIB=lego-slam_amd/lib/liblego_ba_$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ab_$v.log 2>&1 || exit $?
  python3 - "$v" gpurun_out/ab_$v.log >> gpurun_out/ab.log <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l)
        ks = d['kernels_ms_per_solve']
        print(sys.argv[1], d['ms_per_step'], 'k_lin/launch', d['roofline']['avg_launch_ms'], 'trials', d['trials_per_solve'], ks)
PY
done

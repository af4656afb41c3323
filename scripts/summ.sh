# summarise a gpu_round.sh run (host side)
tail -4 gpurun_out/t.log
python3 - <<'PY'
import json
for line in open("gpurun_out/b.log"):
    if line.startswith("{"):
        d = json.loads(line)
        for k in ("value", "ms_per_step", "ms_per_step_with_kernel_events", "iterations_per_solve", "trials_per_solve", "kernels_ms_per_solve", "cpu_baseline", "chi2_rel_vs_oracle", "speedup_vs_cpu", "roofline"):
            print(k, d.get(k))
PY
cat gpurun_out/stamps.log
cut -d, -f1-4 gpurun_out/prof/run_kernel_stats.csv | sed 's/(.*)"/"/'

"""k_lin launch durations from a rocprofv3 --kernel-trace of `bench.py --no-extras` (scripts/gpu_r02.sh
prof stage): the bench's back-to-back replays (its live roofline timing, the last `reps` launches)
and the launches inside the timed solves (after k_ctrl).  Excluded by duration: launches enqueued
past the device's stop (they exit at once, < 10 us) and the final iteration's evaluate-only launches
(ctrl.evo, ~15 us): neither is the per-trial linearisation the roofline prices.  Writes the JSON bench.py reports beside its live
number.
usage: python scripts/rocprof_k_lin.py <kernel_trace.csv> <out.json> <workload key> [reps]
"""
import csv
import json
import sys

path, out, workload = sys.argv[1], sys.argv[2], sys.argv[3]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 50
rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].startswith("void k_lin<3, true, false>")]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0 for r in rows]
replay = dur[-reps:]
solve = [d for d in dur[:-(reps + 1)] if d > 25.0]
res = {"workload": workload, "kernel": "k_lin<3, true, false>", "source": path.split("/")[-1],
       "replay_launches": len(replay), "replay_avg_us": round(sum(replay) / len(replay), 3),
       "in_solve_launches": len(solve), "in_solve_avg_us": round(sum(solve) / len(solve), 3)}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))

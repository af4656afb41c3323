"""Per-kernel average duration over ACTIVE launches from a rocprofv3 kernel trace.

Launches enqueued past the device's stop (the host keeps two trials in flight) exit at their first
instruction and take < 5 us; `--stats` averages them in, this script leaves them out.
usage: python scripts/rocprof_active.py gpurun_out/prof/run_kernel_trace.csv
"""
import csv
import sys

durs = {}
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0]
    durs.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
print(f"{'kernel':28s} {'launches':>8s} {'active':>7s} {'avg_active_us':>14s} {'avg_all_us':>11s}")
for n, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
    a = [x for x in v if x > 5.0]
    aa = sum(a) / len(a) if a else 0.0
    print(f"{n:28s} {len(v):8d} {len(a):7d} {aa:14.2f} {sum(v) / len(v):11.2f}")

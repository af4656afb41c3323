"""Per-kernel durations and inter-kernel gaps of one solve in a rocprofv3 --kernel-trace CSV
(usage: python scripts/trace_gaps.py gpurun_out/trace/run_kernel_trace.csv)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
resets = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("k_reset")]
i0, i1 = resets[-3], resets[-2]          # one whole timed solve (k_reset .. next k_reset)
prev = None
print("one solve(10) of the C3 bench window under rocprofv3 --kernel-trace")
print(f"{'kernel':24s} {'dur us':>8s} {'gap us':>8s}")
last = i0
for i in range(i0, i1):
    r = rows[i]
    if not r["Kernel_Name"].startswith(("k_reset", "void k_lin", "k_reduce", "k_ctrl", "void k_ctrl")):
        break                              # the solve ends at its last controller launch
    last = i
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0.0
    print(f"{r['Kernel_Name'].split('(')[0]:24s} {(e - s) / 1000:8.2f} {gap:8.2f}")
    prev = e
print(f"total {(int(rows[last]['End_Timestamp']) - int(rows[i0]['Start_Timestamp'])) / 1000:.1f} us "
      "(the last launches are trials enqueued past the device's stop: they exit at once)")

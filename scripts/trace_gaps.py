"""Per-kernel durations and inter-kernel gaps of one solve in a rocprofv3 --kernel-trace CSV
(usage: python scripts/trace_gaps.py gpurun_out/trace/run_kernel_trace.csv)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# a solve starts with its initial linearisation (k_lin<T, false, ...>, whose block 0 restarts the solve)
resets = [i for i, r in enumerate(rows) if "k_lin<" in r["Kernel_Name"] and ", false," in r["Kernel_Name"]]
i0, i1 = resets[-3], resets[-2]          # one whole timed solve (initial k_lin .. the next one)
prev = None
print("one solve(10) of the C3 bench window under rocprofv3 --kernel-trace")
print(f"{'kernel':24s} {'dur us':>8s} {'gap us':>8s}")
last = i0
for i in range(i0, i1):
    r = rows[i]
    if not r["Kernel_Name"].startswith(("void k_lin", "k_reduce", "k_ctrl", "void k_ctrl")):
        break                              # the solve ends at its last controller launch
    last = i
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0.0
    print(f"{r['Kernel_Name'].split('(')[0]:24s} {(e - s) / 1000:8.2f} {gap:8.2f}")
    prev = e
print(f"total {(int(rows[last]['End_Timestamp']) - int(rows[i0]['Start_Timestamp'])) / 1000:.1f} us "
      "(the last launches are trials enqueued past the device's stop: they exit at once)")

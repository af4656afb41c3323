"""Per-kernel summary of a rocprofv3 --kernel-trace CSV of scripts/frontend_lk_run.py (the table in
profiles/r0N_rocprof_frontend_lk.txt): launches, mean of the first 20 and the last 3, minimum.

usage: python3 scripts/frontend_prof_summary.py <..._kernel_trace.csv>
"""
import csv
import sys


def main():
    rows = {}
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0]
            if name.startswith("k_frames") or name.startswith("k_lk"):
                rows.setdefault(name, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for name, d in sorted(rows.items()):
        print(f"{name:<12} launches {len(d):>3}  first-20 avg {sum(d[:20]) / len(d[:20]):>9.1f} us  "
              f"last-3 avg {sum(d[-3:]) / len(d[-3:]):>9.1f} us  min {min(d):>8.1f} us")


if __name__ == "__main__":
    main()

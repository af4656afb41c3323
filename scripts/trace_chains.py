"""Per-chain kernel times from a rocprofv3 kernel trace (run_kernel_trace.csv) of LM solves: each chain is
k_lin (trial launch) -> k_reduce -> controller; chains are classed by their k_lin duration (evaluate-only
trials ~15 us at C3, full trials ~40 us, launches past the stop exit at once)."""
import collections
import csv
import sys

import numpy as np

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n_solves = int(sys.argv[2]) if len(sys.argv) > 2 else 0
cut = [float(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "5,25").split(",")]


def kind(n):
    if "k_ctrl" in n:
        return "ctrl"
    if "k_lin<" in n:
        return "lin" if ", true," in n else "init"
    return "red" if "k_reduce" in n else n[:24]


seq = [(kind(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
chains = [(seq[j][1], seq[j + 1][1], seq[j + 2][1]) for j in range(len(seq) - 2)
          if seq[j][0] == "lin" and seq[j + 1][0] == "red" and seq[j + 2][0] == "ctrl"]
lin = np.array([c[0] for c in chains])
for lo, hi, name in ((0, cut[0], "past stop"), (cut[0], cut[1], "evaluate-only"), (cut[1], 1e9, "full")):
    m = (lin >= lo) & (lin < hi)
    if m.sum():
        a = np.array(chains)[m]
        per = f" ({m.sum() / n_solves:.2f} per solve)" if n_solves else ""
        print(f"{name:14s} {m.sum():5d} chains{per}: k_lin {a[:, 0].mean():6.2f}  k_reduce {a[:, 1].mean():5.2f}  "
              f"controller {a[:, 2].mean():6.2f} us")
tot = collections.defaultdict(float)
for k, d in seq:
    tot[k] += d
if n_solves:
    print("per solve (us):", {k: round(v / n_solves, 1) for k, v in tot.items() if k in ("lin", "init", "red", "ctrl")})

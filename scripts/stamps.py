"""Diagnostic: per-phase wave-cycle shares of k_lin / k_ctrl / k_reduce from the
-DLH_STAMPS build (set LH_LIB to lib/liblego_ba_stamps.so).  Shares only — the
stamps perturb scheduling, never quote this build's run time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lego-slam_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import lego_ba  # noqa: E402
from windows import window  # noqa: E402

NAMES = {0: "lin:backsub", 1: "lin:linearize", 2: "lin:Hll+chol", 3: "lin:G+bsd", 4: "lin:pose-tasks",
         5: "lin:G-image", 6: "lin:mfma", 7: "lin:combine", 8: "lin:epilogue barrier", 9: "lin:shfl reductions", 10: "lin:slab write", 11: "ctrl:S+perm+load",
         12: "ctrl:diag tile+factor (w0)", 13: "ctrl:back-subst", 14: "ctrl:poses", 16: "ctrl:LDLT steps", 17: "ctrl:LM logic", 18: "ctrl:block0", 19: "ctrl:commit+dg", 21: "ctrl:rank", 20: "reduce"}

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
w = window(cfg, seed=0, family="stable_noout")
s = lego_ba.Solver(device=0)
s.upload(w)
s.solve_resident()
lego_ba.debug_stamps(reset=True)
n = 5
trials = 0
for _ in range(n):
    trials += s.solve_resident()["trials"] + 1
st = lego_ba.debug_stamps(reset=True)
lin = sum(int(st[i]) for i in range(10))  # 10 is shared with ctrl:dx scatter
ctrl = sum(int(st[i]) for i in range(10, 24) if i != 20)
print(f"{cfg}: {trials} k_lin launches; totals (wave-cycles/launch): lin {lin / trials:.3e} ctrl {ctrl / trials:.3e} reduce {int(st[20]) / trials:.3e}")
for i, nm in NAMES.items():
    v = int(st[i])
    base = lin if i < 10 else (max(v, 1) if i == 20 else ctrl)
    print(f"  {nm:20s} {v / trials:12.3e} wave-cycles/launch  {100.0 * v / max(base, 1):5.1f}%")

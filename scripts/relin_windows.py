"""Checks tests/windows.py RELIN_WINDOWS on the CPU: for each window, the oracle's per-trial accept/reject string
(its verbose-2 log) at 1, 2, 8 and 16 threads and under 1e-12 relative landmark perturbations, and the spread of
every trial's candidate chi2 across those runs.  A window qualifies when the string is the same everywhere and
ends an iteration before the last with an acceptance after a rejection (the GPU then runs a re-linearisation
chain, DESIGN.md 2, whatever its own summation order).  Each run is a subprocess (the oracle prints from C)."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]

CHILD = r"""
import sys, json
sys.path[:0] = [%r, %r]
import numpy as np, oracle_bind as ob
from windows import relin_window
a = json.loads(sys.argv[1])
w = relin_window(a["gen"])
if a["pert"]:
    rng = np.random.default_rng(a["pert"])
    w["lm_xyz"] = w["lm_xyz"] * (1 + 1e-12 * rng.standard_normal(w["lm_xyz"].shape))
ob.solve(w, verbose=2, n_threads=a["th"], max_iters=3, **a["opt"])
""" % (os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python"))


def decisions(gen, opt, th, pert):
    out = subprocess.run([sys.executable, "-c", CHILD, json.dumps(dict(gen=gen, opt=opt, th=th, pert=pert))],
                         capture_output=True, text=True, check=True).stdout
    tr = [ln.split() for ln in out.splitlines() if ln.startswith("trial")]
    return "".join("A" if float(t[2]) > 0 else "R" for t in tr), [float(t[6]) for t in tr]


def main():
    from windows import RELIN_WINDOWS
    ok = True
    for kind, gen, opt, want, _ in RELIN_WINDOWS:
        runs = [decisions(gen, opt, th, pert) for th, pert in ((8, 0), (1, 0), (2, 0), (16, 0), (8, 1), (8, 2))]
        strs = {s for s, _ in runs}
        spread = float(np.max(np.abs(np.array([c for _, c in runs]) / np.array(runs[0][1]) - 1))) if len(strs) == 1 else None
        good = strs == {want}
        ok &= good
        print(f"{kind:28s} {sorted(strs)} spread {spread} {'ok' if good else 'CHANGED'}", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

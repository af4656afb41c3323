"""Per-iteration chi2 and lambda of the headline window and the live configuration (and a few default-family
windows): how small the last accepted decrease is before a solve stalls."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"), os.path.join(os.path.dirname(__file__), "..", "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import lego_ba  # noqa: E402
from windows import window  # noqa: E402

for name, w in (("C3 stable_noout (headline)", window("C3", seed=0, family="stable_noout")),
                ("C3 default (live)", window("C3", seed=0)),
                ("C3 default seed 1", window("C3", seed=1)),
                ("C3 default seed 2", window("C3", seed=2)),
                ("C2 default seed 0", window("C2", seed=0)),
                ("C2 stable seed 1", window("C2", seed=1, family="stable"))):
    s = lego_ba.Solver()
    r = s.solve(w)
    c = np.array(r["trace_chi2"])   # the initial chi2, then each completed iteration's
    rel = -np.diff(c) / c[:-1]
    print(f"{name}: it {r['iterations']} trials {r['trials']} acc {r['accepted']} chains {s.chains()}", flush=True)
    print("   chi2:", " ".join(f"{x:.10g}" for x in c), flush=True)
    print("   rel decrease:", " ".join(f"{x:.2e}" for x in rel), flush=True)
    s.close()

"""Bitwise comparison of two builds of the library (LH_LIB) on the windows whose trajectories are most sensitive
to rounding: the headline C3 window, the live configuration, the gate-1 survey window, a 128-keyframe banded window
and the eval-first windows.  Each build runs in its own process (LH_NO_BATCH=1 in both, so that a change of the
batch path alone does not show); the parent compares every output array.
usage: python3 scripts/lib_bitwise.py OTHER_LIB [THIS_LIB]"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if len(sys.argv) > 2 and sys.argv[1] == "--child":
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
    import numpy as np
    import lego_ba
    from windows import STABLE, window
    out = {}

    def banded(P):
        w = lego_ba.generate_window(P=P, L=50000, k=8, seed=3, **dict(STABLE, outlier_frac=0.0))
        f = np.zeros(P, np.uint8)
        f[0] = 1
        w["pose_fixed"] = f
        return w

    cases = [("headline", window("C3", seed=0, family="stable_noout"), {}),
             ("live", window("C3", seed=0, family="default"), {}),
             ("survey gate 1", window("C3", seed=5, family="default"), dict(gate_mode=1)),
             ("P128", banded(128), {}),
             ("C2", window("C2", seed=0), {}),
             ("C2 fp32", window("C2", seed=0), dict(precision=lego_ba.LH_PREC_FP32_RESID))]
    for name, w, kw in cases:
        r = lego_ba.Solver(**kw).solve(w)
        for k in ("pose_Tcw", "lm_xyz", "edge_robust_chi2"):
            out[f"{name}/{k}"] = r[k]
        out[f"{name}/scalars"] = np.array([r["iterations"], r["trials"], r["chi2_final"]])
    np.savez(sys.argv[2], **out)
    sys.exit(0)

import numpy as np  # noqa: E402

res = []
with tempfile.TemporaryDirectory() as d:
    for lib in (sys.argv[2] if len(sys.argv) > 2 else None, sys.argv[1]):
        env = dict(os.environ, LH_NO_BATCH="1")
        if lib:
            env["LH_LIB"] = lib
        f = os.path.join(d, f"{len(res)}.npz")
        subprocess.run([sys.executable, __file__, "--child", f], env=env, check=True)
        res.append(dict(np.load(f)))
a, b = res
diff = {k: bool(np.array_equal(a[k], b[k])) for k in a}
print(json.dumps({"all_equal": all(diff.values()),
                  "scalars": {k: [a[k].tolist(), b[k].tolist()] for k in a if k.endswith("scalars")},
                  "differ": [k for k, v in diff.items() if not v]}))

"""Batched rejection runs against one rung per chain (LH_NO_BATCH=1), alternated twice in one
process, on the windows that reject: the live configuration, the gate-1 survey window, C4 on one GPU and the
128- / 256-keyframe banded windows.  Prints ms per solve, trials, chains and batches per solve for each.
usage: python3 scripts/batch_ab.py [solves_c3 [window-name filter]]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lego_ba  # noqa: E402
from windows import STABLE, window  # noqa: E402

n_c3 = int(sys.argv[1]) if len(sys.argv) > 1 else 100
only = sys.argv[2] if len(sys.argv) > 2 else ""


def banded(P):
    w = lego_ba.generate_window(P=P, L=50000, k=8, seed=3, **dict(STABLE, outlier_frac=0.0))
    f = np.zeros(P, np.uint8)
    f[0] = 1
    w["pose_fixed"] = f
    return w


cases = [
    ("live C3", lambda: window("C3", seed=0, family="default"), {}, n_c3),
    ("survey C3 gate 1", lambda: window("C3", seed=5, family="default"), dict(gate_mode=1), n_c3),
    ("C4 1 GPU gate 1", lambda: window("C4", seed=0, family="stable_noout"), dict(gate_mode=1), max(5, n_c3 // 10)),
    ("P128 banded", lambda: banded(128), {}, max(5, n_c3 // 10)),
    ("P256 banded", lambda: banded(256), {}, max(5, n_c3 // 20)),
]


def run(w, kw, n, batch):
    if batch:
        os.environ.pop("LH_NO_BATCH", None)
    else:
        os.environ["LH_NO_BATCH"] = "1"
    s = lego_ba.Solver(**kw)
    s.upload(w)
    os.environ.pop("LH_NO_BATCH", None)
    s.solve_resident()
    chains = s.chains()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr = 0
    for _ in range(n):
        tr += s.solve_resident()["trials"]
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    bt = s.batch()
    r = s.solve_resident(want_states=True)
    out = {"ms_per_solve": round(dt * 1e3, 4), "trials": tr / n, "chains": chains, "batch": bt,
           "chi2": r["chi2_final"]}
    s.close()
    return out


for name, mk, kw, n in cases:
    if only and only not in name:
        continue
    w = mk()
    res = {"batch": [], "serial": []}
    for rnd in range(2):
        for b in (True, False):
            res["batch" if b else "serial"].append(run(w, kw, n, b))
    b, s = res["batch"], res["serial"]
    assert all(x["chi2"] == s[0]["chi2"] for x in b + s), name
    mb = min(x["ms_per_solve"] for x in b)
    ms = min(x["ms_per_solve"] for x in s)
    print(json.dumps({"window": name, "ms_batch": [x["ms_per_solve"] for x in b],
                      "ms_serial": [x["ms_per_solve"] for x in s], "speedup": round(ms / mb, 4),
                      "trials": b[0]["trials"], "chains_batch": b[0]["chains"], "chains_serial": s[0]["chains"],
                      "batch": b[0]["batch"]}), flush=True)

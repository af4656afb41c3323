"""Which windows run re-linearisation chains (an evaluate-only trial accepted outside the final iteration):
trials and chains per window of the test's list, plus variants with a small initial lambda (more rejected
Gauss-Newton-like first steps), eval-first on (the default)."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"), os.path.join(os.path.dirname(__file__), "..", "lego-slam_amd", "python")]
import lego_ba  # noqa: E402
from windows import window  # noqa: E402
from test_gpu_parity import EVAL_FIRST_CASES  # noqa: E402


def mk(wargs):
    from windows import multi_camera
    wargs = dict(wargs)
    cams = wargs.pop("cams", 0)
    w = window(wargs.pop("cfg"), seed=wargs.pop("seed")) if "cfg" in wargs else lego_ba.generate_window(k=8, **wargs)
    return multi_camera(w, cams, seed=1) if cams else w


for name, wargs, kw, ctrl in EVAL_FIRST_CASES:
    for extra in ({}, dict(lambda_init=1e-3), dict(lambda_init=1e-1), dict(lambda_init=1e1)):
        s = lego_ba.Solver(**dict(kw, **extra))
        r = s.solve(mk(wargs))
        print(f"{name:16s} {str(extra):24s} {s.controller():9s} it {r['iterations']:2d} trials {r['trials']:3d} "
              f"acc {r['accepted']:2d} chains {s.chains():3d} relin {s.chains() - r['trials']}", flush=True)
        s.close()

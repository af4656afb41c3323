"""Diagnostic for the two-chain k_ctrl schedule: the chaotic outlier windows of the parity suite (the Huber
gate residue, base_edge.cpp:55), solved on the GPU with the two-chain schedule (LH_ND=1) and without (the
one-chain natural order), against the oracle's 16 thread-count outcomes (iterations, trials, final chi2)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import lego_ba      # noqa: E402
import oracle_bind as ob  # noqa: E402
from windows import window  # noqa: E402

cases = [("C1", 1, "stable"), ("mini", 0, "stable"), ("C2", 1, "stable"), ("C2", 2, "stable"), ("C2", 0, "default"),
         ("C2", 1, "default"), ("mini", 3, "default")]
for cfg, seed, fam in cases:
    w = window(cfg, seed=seed, family=fam)
    runs = [ob.solve(w, n_threads=t) for t in range(1, 17)]
    outs = sorted({(r["iterations"], r["trials"], round(r["chi2_final"], 6)) for r in runs})
    line = [f"{cfg}-{seed}-{fam} P={len(w['pose_Tcw'])}"]
    for nd in (True, False):
        if nd:
            os.environ["LH_ND"] = "1"
        else:
            os.environ.pop("LH_ND", None)
        s = lego_ba.Solver()
        g = s.solve(w)
        s.close()
        best = min(abs(g["chi2_final"] - r["chi2_final"]) / r["chi2_final"] for r in runs)
        line.append(f"{'nd' if nd else 'nat'}: it {g['iterations']} tr {g['trials']} chi2 {g['chi2_final']:.9g} "
                    f"best rel {best:.2e}")
    os.environ.pop("LH_ND", None)
    print(" | ".join(line), "| oracle outcomes", outs[:6], flush=True)

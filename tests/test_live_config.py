"""The reference's live configuration at the headline size: survey-default C3 (20 KF / 50 k landmarks /
400 k observations, free gauge, left image only, 2 % outliers; backend_lego.cpp:67-79, 92-94), solved
on the GPU through the C ABI and held against the oracle re-run over OpenMP thread counts 1-16.

With the reference Huber gate (base_edge.cpp:55) no such window is reproducible by the reference
itself: every thread count of the oracle lands on its own outcome (seeds 0-3, 1-8 threads: 32 runs,
32 distinct (iterations, trials, chi2), 1e-4..1e-3 apart).  The runs agree to ~1e-11 through trace
entry 1 (the chi2 after the first iteration) and part at entry 2, by 1e-3..1e-2: after the first
step the outlier edges' gate residues (analytically zero) take the signs of their rounding, and
the second linearisation weights them differently.  With the residue taken as 0 on both sides
(gate_mode 1) the same runs agree to ~1e-10 through entry 4.  So:
  * gate 0: the GPU must agree with the oracle where the oracle agrees with itself (the trace
    prefix before its own split, at the oracle's own spread), part where it parts, and end inside
    the oracle's 16-outcome envelope;
  * gate 1: the GPU must match one of the oracle's own 16 outcomes: the same iterations and
    trials, final chi2 within 1e-6 (the north-star bar).
"""
import numpy as np
import pytest

import lego_ba
import oracle_bind as ob
from windows import window

pytestmark = pytest.mark.gpu

THREADS = range(1, 17)


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


def _oracle_runs(w, **opt):
    return [ob.solve(w, n_threads=t, **opt) for t in THREADS]


def _split_index(runs, tol):
    """First trace entry where the oracle's own runs differ by more than tol (relative)."""
    n = min(len(r["trace_chi2"]) for r in runs)
    for k in range(n):
        v = [r["trace_chi2"][k] for r in runs]
        if (max(v) - min(v)) / min(v) > tol:
            return k
    return n


@pytest.fixture(scope="module")
def c3_default():
    w = window("C3", seed=0)
    assert w.get("pose_fixed") is None and not np.any(w["obs_cam"])        # gauge free, left image only
    assert len(w["obs_pose"]) == 400_000 and len(w["lm_xyz"]) == 50_000
    return w


def test_c3_live_config_reference_gate(c3_default):
    w = c3_default
    runs = _oracle_runs(w)
    outcomes = {(r["iterations"], r["trials"], round(r["chi2_final"], 3)) for r in runs}
    g = lego_ba.Solver().solve(w)
    # where the oracle agrees with itself, the GPU agrees with it at the oracle's own spread
    k_split = _split_index(runs, 1e-9)
    assert k_split == 2, f"the oracle's runs part at trace entry {k_split}"
    o = runs[0]
    assert rel(g["chi2_initial"], o["chi2_initial"]) < 1e-12
    assert rel(g["trace_lambda"][0], o["trace_lambda"][0]) < 1e-12
    assert rel(g["trace_chi2"][1], o["trace_chi2"][1]) < 1e-9
    assert rel(g["trace_lambda"][1], o["trace_lambda"][1]) < 1e-9
    # ... and from there the reference lands on a different outcome per summation order: the GPU's
    # final chi2 lies inside the envelope of the oracle's 16 outcomes, its iteration count in range
    chis = [r["chi2_final"] for r in runs]
    its = [r["iterations"] for r in runs]
    assert len(outcomes) >= 8     # the finding this test documents: no reproducible outcome to match
    assert min(chis) * (1 - 1e-6) <= g["chi2_final"] <= max(chis) * (1 + 1e-6)
    assert min(its) <= g["iterations"] <= max(its)
    assert np.all(np.diff(g["trace_chi2"][:g["iterations"] + 1]) <= 0)


def test_c3_live_config_gate_residue_zero_matches_an_oracle_outcome(c3_default):
    w = c3_default
    runs = _oracle_runs(w, gate_mode=1)
    g = lego_ba.Solver(gate_mode=1).solve(w)
    assert _split_index(runs, 1e-9) >= 4          # reproducible well past where gate 0 parts
    same = [r for r in runs if (r["iterations"], r["trials"]) == (g["iterations"], g["trials"])]
    assert same, f"GPU {g['iterations']}/{g['trials']} is none of the oracle's outcomes"
    best = min(rel(g["chi2_final"], r["chi2_final"]) for r in same)
    assert best < 1e-6, f"closest same-path oracle outcome {best:.2e}"
    o = same[0]
    assert rel(g["chi2_initial"], o["chi2_initial"]) < 1e-12
    k = _split_index(runs, 1e-9)
    assert np.allclose(g["trace_chi2"][:k], o["trace_chi2"][:k], rtol=1e-9, atol=0)

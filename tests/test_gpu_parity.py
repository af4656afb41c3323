"""GPU parity tests: the HIP solver (liblego_ba.so, through the C ABI) against
the oracle (oracle/lego_oracle.c) on the same seeded windows.

Tolerances (north star: final chi2 within 1e-6 relative):
  * one LM trial (per-linearisation arithmetic, any window): chi2 1e-12 / 1e-10,
    states 1e-9 — the kernels and the oracle compute the same numbers up to
    summation order;
  * full solve on "stable" windows (oracle reproducible under reordering):
    chi2 <= 1e-6, identical iteration / trial counts;
  * full solve on the survey-default (chaotic) windows: within the oracle's
    own reorder spread (see tests/windows.py).
"""
import ctypes as C

import numpy as np
import pytest

import lego_ba
import oracle_bind as ob
from align import aligned_errors, oracle_state_spread
from windows import window

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solver():
    s = lego_ba.Solver()
    yield s
    s.close()


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


def test_mfma_f64_accumulator_layout():
    import torch
    lib = lego_ba.ba_lib()
    lib.lh_debug_mfma_probe.argtypes = [C.c_void_p] * 3
    # exact small-integer data (every product and partial sum representable): layout, not rounding
    A = (torch.arange(64, dtype=torch.float64, device="cuda").reshape(16, 4) % 7) - 3
    B = ((torch.arange(64, dtype=torch.float64, device="cuda").reshape(4, 16) ** 2) % 11) - 5   # asymmetric
    D = torch.zeros(16, 16, dtype=torch.float64, device="cuda")
    assert lib.lh_debug_mfma_probe(A.data_ptr(), B.data_ptr(), D.data_ptr()) == 0
    assert torch.equal(D, A @ B)


def _ldlt_probe(S, b):
    import torch
    lib = lego_ba.ba_lib()
    lib.lh_debug_ldlt_probe.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    St = torch.tensor(S, dtype=torch.float64, device="cuda").contiguous()
    bt = torch.tensor(b, dtype=torch.float64, device="cuda")
    xt = torch.zeros(len(b), dtype=torch.float64, device="cuda")
    assert lib.lh_debug_ldlt_probe(St.data_ptr(), bt.data_ptr(), len(b), xt.data_ptr()) == 0
    return xt.cpu().numpy()


@pytest.mark.parametrize("n", [6, 12, 60, 96, 114, 120, 126, 132, 186, 258, 384])
def test_reduced_solve_spd(n):
    """k_ctrl's blocked LDL^T + solve (through the test hook) against numpy on SPD systems
    shaped like S + lambda I (problem.cpp:404-420): block-banded, wide diagonal spread.  Past 128
    rows (windows past 21 poses) the hook runs k_ctrl_g's global-memory solve."""
    rng = np.random.default_rng(n)
    P = n // 6
    S = np.zeros((n, n))
    for p in range(P):
        for q in range(p, min(P, p + 8)):
            B = rng.standard_normal((6, 6)) * (10.0 ** rng.uniform(0, 4))
            S[6 * p:6 * p + 6, 6 * q:6 * q + 6] += B
    S = S @ S.T + np.diag(10.0 ** rng.uniform(2, 9, n))
    b = rng.standard_normal(n) * 1e3
    x = _ldlt_probe(S, b)
    xr = np.linalg.solve(S, b)
    assert np.linalg.norm(x - xr) <= 1e-10 * np.linalg.norm(xr)


@pytest.mark.parametrize("n", [60, 222])
def test_reduced_solve_zero_rows(n):
    """STRATEGY1 with a fixed pose: exactly-zero rows and columns (diag 0 + lambda*0); Eigen's
    LDLT pivots them last, skips the invalid pivots and returns 0 there (LDLT::_solve_impl)."""
    rng = np.random.default_rng(7)
    M = rng.standard_normal((n, n))
    S = M @ M.T + n * np.eye(n)
    S[:6, :] = 0.0
    S[:, :6] = 0.0
    b = rng.standard_normal(n)
    b[:6] = 0.0
    x = _ldlt_probe(S, b)
    assert np.all(x[:6] == 0.0)
    xr = np.linalg.solve(S[6:, 6:], b[6:])
    assert np.allclose(x[6:], xr, rtol=1e-11, atol=1e-13)


@pytest.mark.parametrize("n", [138, 240, 384])
def test_reduced_solve_global_vs_oracle(n):
    """k_ctrl_g's solve against the oracle's restatement of Eigen's LDLT (ldlt_solve: the same
    pivot order, the same triangular-solve order); only the factor's rounding differs."""
    rng = np.random.default_rng(100 + n)
    M = rng.standard_normal((n, n))
    S = M @ M.T + np.diag(10.0 ** rng.uniform(0, 6, n))
    b = rng.standard_normal(n)
    x = _ldlt_probe(S, b)
    xo = ob.ldlt_solve(S, b)
    assert np.linalg.norm(x - xo) <= 1e-11 * np.linalg.norm(xo)


@pytest.mark.parametrize("cfg,seed,family", [("C1", 0, "default"), ("C1", 1, "stable"), ("mini", 0, "default"),
                                              ("C2", 0, "default"), ("C2", 1, "stable")])
def test_single_trial_parity(solver, cfg, seed, family):
    w = window(cfg, seed=seed, family=family)
    g = lego_ba.Solver(max_iters=1, max_trials=1).solve(w)
    o = ob.solve(w, max_iters=1, max_trials=1)
    assert g["trials"] == o["trials"] == 1 and g["accepted"] == o["accepted"]
    assert rel(g["chi2_initial"], o["chi2_initial"]) < 1e-12
    assert rel(g["trace_lambda"][0], o["trace_lambda"][0]) < 1e-12
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-9
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-9)
    assert np.allclose(g["lm_xyz"], o["lm_xyz"], atol=1e-7)
    assert np.allclose(g["edge_robust_chi2"], o["edge_robust_chi2"], rtol=1e-8, atol=1e-9)


def oracle_envelope(w, threads=(1, 2, 8), **opt):
    """The oracle re-run with different summation orders: its own final-chi2 spread."""
    runs = [ob.solve(w, n_threads=t, **opt) for t in threads]
    chis = [r["chi2_final"] for r in runs]
    return runs[0], (max(chis) - min(chis)) / min(chis), {r["iterations"] for r in runs}


@pytest.mark.parametrize("cfg,seed", [("C1", 0), ("C1", 2), ("mini", 1), ("C2", 0), ("C2", 1)])
def test_initial_edge_chi2_bitwise(solver, cfg, seed):
    # residual, robust weight and rho0 are a bitwise mirror of the oracle's Eigen/Sophus restatement
    w = window(cfg, seed=seed)
    g = lego_ba.Solver(max_iters=0).solve(w)
    o = ob.solve(w, max_iters=0)
    assert np.array_equal(g["edge_robust_chi2"], o["edge_robust_chi2"])
    assert rel(g["chi2_initial"], o["chi2_initial"]) < 1e-13


@pytest.mark.parametrize("cfg,seed", [("C1", 0), ("C1", 1), ("mini", 0), ("mini", 1), ("C2", 0), ("C2", 1),
                                      ("C2", 2), ("C2", 3)])
def test_full_solve_parity_stable(solver, cfg, seed):
    """North-star bar (final chi2 within 1e-6) on windows whose reference trajectory is
    reproducible: the oracle's final chi2 moves < 1e-12 across summation orders."""
    w = window(cfg, seed=seed, family="stable_noout")
    o, spread, its = oracle_envelope(w, threads=(1, 2, 8, 16))
    assert spread < 1e-12, f"window not reproducible under reordering (spread {spread:.1e})"
    g = solver.solve(w)
    assert g["iterations"] in its
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-6
    assert rel(g["trace_chi2"][1], o["trace_chi2"][1]) < 1e-9      # after the first (bitwise-linearised) step
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-6)
    assert np.allclose(g["lm_xyz"], o["lm_xyz"], atol=1e-6)


@pytest.mark.parametrize("cfg,seed", [("C1", 1), ("mini", 0), ("C2", 1), ("C2", 2)])
def test_full_solve_outlier_window_within_oracle_envelope(solver, cfg, seed):
    """Windows with outliers: the Huber gate (base_edge.cpp:55) tests the sign of a rounding
    residue on every outlier edge, so the reference itself lands in different basins under
    summation reorders (e.g. C2 seed 1: 10 iterations for 14 of 16 thread counts, a 3-iteration
    stall for the other two).  The GPU must match one of the oracle's own outcomes to 1e-6."""
    w = window(cfg, seed=seed, family="stable")
    runs = [ob.solve(w, n_threads=t) for t in range(1, 17)]
    g = solver.solve(w)
    assert min(rel(g["chi2_final"], r["chi2_final"]) for r in runs) < 1e-6
    assert rel(g["trace_chi2"][1], runs[0]["trace_chi2"][1]) < 1e-9


@pytest.mark.parametrize("cfg,seed", [("C2", 0), ("C2", 1), ("mini", 3)])
def test_full_solve_default_window_within_oracle_envelope(solver, cfg, seed):
    """Survey-default windows: the reference LM is chaotic under reordering (Huber gate,
    base_edge.cpp:55); the GPU must land inside the oracle's own reorder envelope."""
    w = window(cfg, seed=seed)
    o, spread, _ = oracle_envelope(w)
    g = solver.solve(w)
    assert rel(g["chi2_final"], o["chi2_final"]) <= max(1e-6, 10 * spread)
    assert g["chi2_final"] < g["chi2_initial"]
    assert rel(g["trace_chi2"][0], o["trace_chi2"][0]) < 1e-13
    assert rel(g["trace_lambda"][0], o["trace_lambda"][0]) < 1e-12


def test_deterministic_and_resident_restart(solver):
    w = window("C2", seed=3)
    a = solver.solve(w)
    solver.upload(w)
    b = solver.solve_resident(want_states=True, want_edges=True)
    c = solver.solve_resident(want_states=True, want_edges=True)
    for k in ("pose_Tcw", "lm_xyz", "edge_robust_chi2"):
        assert np.array_equal(a[k], b[k]) and np.array_equal(b[k], c[k])
    assert a["chi2_final"] == b["chi2_final"] == c["chi2_final"]


def test_observation_order_is_free(solver):
    w = window("mini", seed=2)
    perm = np.random.default_rng(0).permutation(len(w["obs_pose"]))
    w2 = dict(w)
    for k in ("obs_pose", "obs_lm", "obs_cam", "obs_uv"):
        w2[k] = w[k][perm]
    a, b = solver.solve(w), solver.solve(w2)
    assert a["chi2_final"] == b["chi2_final"]
    assert np.array_equal(a["edge_robust_chi2"][perm], b["edge_robust_chi2"])


@pytest.mark.parametrize("cfg,seed", [("C1", 0), ("mini", 1)])
def test_strategy1_single_trial_parity(cfg, seed):
    w = window(cfg, seed=seed, family="stable")
    g = lego_ba.Solver(strategy=1, max_iters=1, max_trials=1).solve(w)
    o = ob.solve(w, strategy=1, max_iters=1, max_trials=1)
    assert g["accepted"] == o["accepted"]
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-9
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-9)


def test_strategy1_parity():
    w = window("C1", seed=1, family="stable")
    o, spread, its = oracle_envelope(w, strategy=1)
    g = lego_ba.Solver(strategy=1).solve(w)
    assert rel(g["chi2_final"], o["chi2_final"]) < max(1e-6, 10 * spread)
    # STRATEGY1 drives lambda to its 1e-7 floor (Gauss-Newton); the last decrements sit
    # within a few 1e-5 of the absolute stop threshold (problem.cpp:210), where the
    # oracle's own iteration count moves with the summation order (7 or 8 on C1 seed 0)
    assert min(its) - 1 <= g["iterations"] <= max(its) + 1


def test_no_robust_kernel_and_lambda_init():
    w = window("C1", seed=0, family="stable_noout")
    g = lego_ba.Solver(huber_delta=0.0, lambda_init=10.0).solve(w)
    o = ob.solve(w, huber_delta=0.0, lambda_init=10.0)
    assert g["trace_lambda"][0] == 10.0
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-8


def test_fixed_pose_and_unobserved_landmark(solver):
    w = window("C1", seed=1, family="stable")
    w["lm_xyz"] = np.vstack([w["lm_xyz"], [[1.0, 2.0, 3.0]]])   # landmark with no edge: not a vertex
    g = solver.solve(w)
    assert np.allclose(g["pose_Tcw"][0], w["pose_Tcw"][0], atol=1e-12)
    assert np.array_equal(g["lm_xyz"][-1], [1.0, 2.0, 3.0])


def test_error_paths(solver):
    w = window("C1")
    empty = dict(w, obs_pose=w["obs_pose"][:0], obs_lm=w["obs_lm"][:0], obs_cam=w["obs_cam"][:0], obs_uv=w["obs_uv"][:0])
    with pytest.raises(lego_ba.LhError) as e:
        solver.solve(empty)
    assert e.value.status == lego_ba.LH_E_EMPTY
    bad = dict(w, obs_pose=w["obs_pose"].copy())
    bad["obs_pose"][0] = 99
    with pytest.raises(lego_ba.LhError) as e:
        solver.solve(bad)
    assert e.value.status == lego_ba.LH_E_BADARG
    dup = dict(w)
    for k in ("obs_pose", "obs_lm", "obs_cam", "obs_uv"):
        dup[k] = np.concatenate([w[k], w[k][:1]])
    with pytest.raises(lego_ba.LhError) as e:
        solver.solve(dup)
    assert e.value.status == lego_ba.LH_E_UNSUPPORTED


def test_outlier_pass_on_solver_output(solver):
    w = window("mini", seed=0, family="stable")
    g = solver.solve(w)
    o = ob.solve(w)
    fg, thg, _, _ = lego_ba.classify_outliers(g["edge_robust_chi2"])
    fo, tho, _, _ = lego_ba.classify_outliers(o["edge_robust_chi2"])
    assert thg == tho
    assert np.mean(fg != fo) < 1e-3


def test_c3_window_parity_and_properties():
    """C3 with 2 % outliers.  With the reference Huber gate its trajectory is chaotic even for the
    oracle (4 / 8 / 5 OpenMP threads: 8 / 10 / 7 iterations, final chi2 1e-4 apart): the solve
    must land in that envelope.  With the gate's rounding residue taken as 0 (gate_mode 1) the
    oracle is reproducible to 1e-14 and the GPU is held to the north-star bar."""
    w = window("C3", seed=0, family="stable")
    g1 = lego_ba.Solver(gate_mode=1).solve(w)
    o1, spread1, its1 = oracle_envelope(w, threads=(4, 8), gate_mode=1)
    assert spread1 < 1e-12 and its1 == {g1["iterations"]} and g1["trials"] == o1["trials"]
    assert rel(g1["chi2_final"], o1["chi2_final"]) < 1e-6
    assert np.allclose(g1["pose_Tcw"], o1["pose_Tcw"], atol=1e-6)
    g = lego_ba.Solver().solve(w)
    o, spread, its = oracle_envelope(w, threads=(4, 8, 5))
    assert min(its) - 1 <= g["iterations"] <= max(its) + 1
    assert rel(g["chi2_final"], o["chi2_final"]) < max(1e-5, 10 * spread)
    # size-independent properties
    assert np.all(np.diff(g["trace_chi2"]) <= 0)
    assert np.all(np.isfinite(g["lm_xyz"])) and np.all(np.isfinite(g["pose_Tcw"]))
    R = g["pose_Tcw"].reshape(-1, 3, 4)[:, :, :3]
    assert np.allclose(R @ R.transpose(0, 2, 1), np.eye(3), atol=1e-12)


def test_rccl_data_path_one_rank(monkeypatch):
    """The multi-GPU data path (an RCCL all-reduce of the packed reduced system per trial, a MAX
    all-reduce of max|H_ll diag| at the initial linearisation) on a one-rank communicator: the
    collectives, their buffers and stream order run, and the result is bit-identical."""
    w = window("C2", seed=0, family="stable_noout")
    a = lego_ba.Solver().solve(w)
    monkeypatch.setenv("LH_FORCE_RCCL", "1")
    b = lego_ba.Solver().solve(w)
    assert a["chi2_final"] == b["chi2_final"] and a["iterations"] == b["iterations"]
    assert np.array_equal(a["pose_Tcw"], b["pose_Tcw"]) and np.array_equal(a["lm_xyz"], b["lm_xyz"])


@pytest.mark.parametrize("kmin,kmax", [(3, 10), (2, 6)])
def test_random_pose_subsets_all_tile_counts(kmin, kmax):
    """Landmarks seen by random subsets of 2..10 keyframes: chunks with T = 1..4 MFMA tiles
    (one k_lin launch per T), windows unions up to 10 poses, sub-batches with 2..16-lane groups."""
    w = window("C2", seed=3, family="stable_noout", pose_mode=1, k_min=kmin, k_max=kmax)
    g = lego_ba.Solver(max_iters=1, max_trials=1).solve(w)
    o = ob.solve(w, max_iters=1, max_trials=1)
    assert rel(g["chi2_initial"], o["chi2_initial"]) < 1e-12
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-9
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-9)
    assert np.allclose(g["lm_xyz"], o["lm_xyz"], atol=1e-7)
    gf = lego_ba.Solver().solve(w)
    of, spread, its = oracle_envelope(w, threads=(1, 2, 8))
    assert rel(gf["chi2_final"], of["chi2_final"]) < max(1e-6, 10 * spread)


def test_largest_lds_window_p21():
    """P = 21 keyframes: the largest reduced system k_ctrl factors in LDS (126 x 126, two
    identity padding rows)."""
    w = lego_ba.generate_window(P=21, L=3000, k=8, seed=4, **dict(__import__("windows").STABLE, outlier_frac=0.0))
    f = np.zeros(21, np.uint8)
    f[0] = 1
    w["pose_fixed"] = f
    g = lego_ba.Solver().solve(w)
    o, spread, its = oracle_envelope(w, threads=(1, 2, 8))
    assert g["iterations"] in its
    assert rel(g["chi2_final"], o["chi2_final"]) < max(1e-6, 10 * spread)


def _stable_window(P, L, seed, **kw):
    w = lego_ba.generate_window(P=P, L=L, k=8, seed=seed, **dict(__import__("windows").STABLE, outlier_frac=0.0), **kw)
    f = np.zeros(P, np.uint8)
    f[0] = 1
    w["pose_fixed"] = f
    return w


@pytest.mark.parametrize("P,L,seed,mode", [(22, 3000, 4, 0), (32, 4000, 1, 0), (40, 3000, 3, 1), (64, 6000, 2, 0)])
def test_large_windows_global_memory_solve(P, L, seed, mode):
    """Windows past 21 keyframes (the reference solver takes any number, problem.cpp:277-279).
    Sliding-window structure (mode 0: landmarks seen by runs of 8 consecutive keyframes) gives a
    banded reduced system, factored by k_ctrl_b; mode 1 (landmarks seen by random keyframe subsets:
    chunk windows of several tile counts, a dense reduced system) by k_ctrl_g in global memory.  One
    trial at the single-trial bar, then the full solve at the north-star bar (chi2 1e-6, poses and
    landmarks 1e-6) against the oracle on reproducible windows."""
    kw = dict(pose_mode=1, k_min=2, k_max=8) if mode else {}
    w = _stable_window(P, L, seed, **kw)
    s1 = lego_ba.Solver(max_iters=1, max_trials=1)
    g = s1.solve(w)
    assert s1.controller() == ("k_ctrl_g" if mode else "k_ctrl_b")
    o = ob.solve(w, max_iters=1, max_trials=1)
    assert rel(g["chi2_initial"], o["chi2_initial"]) < 1e-12
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-9
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-9)
    assert np.allclose(g["lm_xyz"], o["lm_xyz"], atol=1e-7)
    gf = lego_ba.Solver().solve(w)
    of, spread, its = oracle_envelope(w, threads=(1, 2, 8))
    assert gf["iterations"] in its
    assert rel(gf["chi2_final"], of["chi2_final"]) < max(1e-6, 10 * spread)
    assert np.allclose(gf["pose_Tcw"], of["pose_Tcw"], atol=1e-6)
    assert np.allclose(gf["lm_xyz"], of["lm_xyz"], atol=1e-6)


@pytest.mark.parametrize("P,L,seed", [(96, 6000, 1), (128, 8000, 1), (128, 8000, 3), (256, 12000, 1)])
def test_banded_ldlt_past_64_keyframes(P, L, seed):
    """The reference's live solver (LDL^T, problem.cpp:420) on windows of 96 to 256 keyframes: the banded
    controller (k_ctrl_b) streams the band of S through one CU's LDS.  One trial at the single-trial
    bar, the full solve at the north-star bar against the oracle's LDLT (windows the oracle reproduces
    across thread counts)."""
    w = _stable_window(P, L, seed)
    s1 = lego_ba.Solver(max_iters=1, max_trials=1)
    g = s1.solve(w)
    assert s1.controller() == "k_ctrl_b"
    o = ob.solve(w, max_iters=1, max_trials=1)
    assert rel(g["chi2_initial"], o["chi2_initial"]) < 1e-12
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-9
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-9)
    assert np.allclose(g["lm_xyz"], o["lm_xyz"], atol=1e-7)
    gf = lego_ba.Solver().solve(w)
    of, spread, its = oracle_envelope(w, threads=(1, 8))
    assert spread < 1e-12
    assert gf["iterations"] == of["iterations"] and gf["trials"] == of["trials"]
    assert rel(gf["chi2_final"], of["chi2_final"]) < 1e-6
    assert np.allclose(gf["pose_Tcw"], of["pose_Tcw"], atol=1e-6)
    assert np.allclose(gf["lm_xyz"], of["lm_xyz"], atol=1e-6)


def test_banded_back_substitution_row_windows(monkeypatch):
    """k_ctrl_b's back substitution holds one row per lane when every row's envelope starts within 56 rows of
    its 8-row block (8-keyframe runs: 47 rows), two rows per lane otherwise.  A row takes the same products
    in the same order either way, so on a narrow window the two forms agree bitwise (LH_NO_NARROW=1 forces
    the two-row form)."""
    w = _stable_window(128, 8000, 3)
    s = lego_ba.Solver()
    a = s.solve(w)
    assert s.controller() == "k_ctrl_b" and s.band_narrow()
    monkeypatch.setenv("LH_NO_NARROW", "1")
    t = lego_ba.Solver()
    b = t.solve(w)
    assert t.controller() == "k_ctrl_b" and not t.band_narrow()
    assert a["iterations"] == b["iterations"] and a["trials"] == b["trials"]
    assert a["chi2_final"] == b["chi2_final"]
    assert np.array_equal(a["pose_Tcw"], b["pose_Tcw"]) and np.array_equal(a["lm_xyz"], b["lm_xyz"])
    s.close()
    t.close()


@pytest.mark.parametrize("P,L,k,seed", [(96, 6000, 11, 1), (128, 50000, 8, 3)])
def test_band_image_equals_packed_blocks(P, L, k, seed, monkeypatch):
    """k_reduce writes a one-rank banded window's S straight into k_ctrl_b's loader order (the band image); the
    loaders then read each element with one load instead of a block-index round trip and a value load.  The
    values and their arithmetic are the same, so the solve is bitwise the one over the packed blocks
    (LH_NO_BIMG=1), rejected trials (the committed image) included."""
    w = lego_ba.generate_window(P=P, L=L, k=k, seed=seed, **dict(__import__("windows").STABLE, outlier_frac=0.0))
    w["pose_fixed"] = np.eye(1, P, dtype=np.uint8)[0]
    s = lego_ba.Solver()
    a = s.solve(w)
    assert s.controller() == "k_ctrl_b"
    monkeypatch.setenv("LH_NO_BIMG", "1")
    t = lego_ba.Solver()
    b = t.solve(w)
    assert a["trials"] > a["iterations"] or P == 96   # the P = 128 window rejects trials: the committed image is read
    assert a["iterations"] == b["iterations"] and a["trials"] == b["trials"]
    assert a["chi2_final"] == b["chi2_final"]
    assert np.array_equal(a["pose_Tcw"], b["pose_Tcw"]) and np.array_equal(a["lm_xyz"], b["lm_xyz"])
    s.close()
    t.close()


@pytest.mark.parametrize("k", [11, 15])
def test_banded_ldlt_wide_band(k):
    """Banded windows whose landmarks span 11 and 15 keyframes (15: the reference's window length, map.h:82):
    rows reach 60-95 columns back, past the one-row-per-lane back substitution's 56, so k_ctrl_b holds two rows
    per lane; 15-keyframe runs make 16-pose chunk windows and steps of 13 units, which the stream loaders
    share.  One trial at the single-trial bar, the full solve against the oracle's LDLT."""
    w = lego_ba.generate_window(P=96, L=6000, k=k, seed=2, **dict(__import__("windows").STABLE, outlier_frac=0.0))
    f = np.zeros(96, np.uint8)
    f[0] = 1
    w["pose_fixed"] = f
    s1 = lego_ba.Solver(max_iters=1, max_trials=1)
    g = s1.solve(w)
    assert s1.controller() == "k_ctrl_b" and not s1.band_narrow() and s1.band_loader_units() == (k == 15)
    o = ob.solve(w, max_iters=1, max_trials=1)
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-9
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-9)
    assert np.allclose(g["lm_xyz"], o["lm_xyz"], atol=1e-7)
    gf = lego_ba.Solver().solve(w)
    of, spread, its = oracle_envelope(w, threads=(1, 8))
    assert gf["iterations"] in its
    assert rel(gf["chi2_final"], of["chi2_final"]) < max(1e-6, 10 * spread)
    assert np.allclose(gf["pose_Tcw"], of["pose_Tcw"], atol=1e-6)
    assert np.allclose(gf["lm_xyz"], of["lm_xyz"], atol=1e-6)


def test_large_window_strategy1():
    """STRATEGY1 (lambda scaled by the diagonal, problem.cpp:420) on a 32-keyframe window: one trial
    at the single-trial bar, the full solve inside the oracle's envelope."""
    w = window("W32", seed=2, family="stable_noout")
    g = lego_ba.Solver(strategy=1, max_iters=1, max_trials=1).solve(w)
    o = ob.solve(w, strategy=1, max_iters=1, max_trials=1)
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-9
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-9)
    gf = lego_ba.Solver(strategy=1).solve(w)
    of, spread, its = oracle_envelope(w, threads=(1, 2, 8), strategy=1)
    assert rel(gf["chi2_final"], of["chi2_final"]) < max(1e-6, 10 * spread)


def test_large_window_default_family_gate1():
    """A survey-default (gauge-free, outliers, left-only) window of 30 keyframes in the diagnostic
    gate mode: inside the oracle's own reorder envelope."""
    w = lego_ba.generate_window(P=30, L=3000, k=8, seed=5)
    g = lego_ba.Solver(gate_mode=1).solve(w)
    o, spread, _ = oracle_envelope(w, threads=(1, 2, 8), gate_mode=1)
    assert rel(g["chi2_final"], o["chi2_final"]) <= max(1e-6, 10 * spread)
    assert g["chi2_final"] < g["chi2_initial"]


def test_window_envelope_edges():
    """Past 64 keyframes LDLT runs when the reduced system is banded (k_ctrl_b); a window whose S is not
    (landmarks coupling keyframes 40 apart) is refused there (the dense k_ctrl_g stops at 64; PCG takes
    it, tests/test_pcg.py); past 256 keyframes nothing is."""
    w = lego_ba.generate_window(P=65, L=500, k=8, seed=4)
    s = lego_ba.Solver(max_iters=1)
    s.solve(w)
    assert s.controller() == "k_ctrl_b"
    L = len(w["lm_xyz"])
    wide = dict(w, lm_xyz=np.vstack([w["lm_xyz"], w["lm_xyz"][:20]]))
    wide["obs_pose"] = np.concatenate([w["obs_pose"], np.tile([0, 40], 20)]).astype(w["obs_pose"].dtype)
    wide["obs_lm"] = np.concatenate([w["obs_lm"], np.repeat(np.arange(L, L + 20), 2)]).astype(w["obs_lm"].dtype)
    wide["obs_cam"] = np.concatenate([w["obs_cam"], np.zeros(40, w["obs_cam"].dtype)])
    wide["obs_uv"] = np.vstack([w["obs_uv"], w["obs_uv"][:40]])
    with pytest.raises(lego_ba.LhError) as e:
        lego_ba.Solver().solve(wide)
    assert e.value.status == lego_ba.LH_E_UNSUPPORTED
    w = lego_ba.generate_window(P=256, L=500, k=8, seed=4)
    w["pose_Tcw"] = np.vstack([w["pose_Tcw"], w["pose_Tcw"][-1:]])
    w["n_poses"] = 257
    with pytest.raises(lego_ba.LhError) as e:
        lego_ba.Solver(linear_solver=lego_ba.LH_SOLVER_PCG).solve(w)
    assert e.value.status == lego_ba.LH_E_UNSUPPORTED


@pytest.mark.parametrize("kmin,kmax,mode", [(11, 16, 1), (2, 16, 1), (8, 15, 0)])
def test_wide_landmarks_up_to_16_poses(kmin, kmax, mode):
    """Landmarks seen by up to 16 keyframes (the reference window is 15 keyframes, map.h:82, so a
    landmark can be seen by all of them): chunk windows of T = 5 and 6 MFMA tiles (k_lin<5>,
    k_lin<6>), slots up to 15, lane groups of 16."""
    p = dict(__import__("windows").STABLE, outlier_frac=0.0)
    w = lego_ba.generate_window(P=20, L=3000, k=kmin, k_max=kmax, seed=2, pose_mode=mode, **p)
    f = np.zeros(20, np.uint8)
    f[0] = 1
    w["pose_fixed"] = f
    g = lego_ba.Solver(max_iters=1, max_trials=1).solve(w)
    o = ob.solve(w, max_iters=1, max_trials=1)
    assert rel(g["chi2_initial"], o["chi2_initial"]) < 1e-12
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-9
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-9)
    assert np.allclose(g["lm_xyz"], o["lm_xyz"], atol=1e-7)
    gf = lego_ba.Solver().solve(w)
    of, spread, its = oracle_envelope(w, threads=(1, 2, 8))
    assert gf["iterations"] in its
    assert rel(gf["chi2_final"], of["chi2_final"]) < max(1e-6, 10 * spread)


def test_landmark_seen_by_17_poses_is_unsupported():
    w = lego_ba.generate_window(P=20, L=200, k=17, seed=1, pose_mode=1)
    with pytest.raises(lego_ba.LhError) as e:
        lego_ba.Solver().solve(w)
    assert e.value.status == lego_ba.LH_E_UNSUPPORTED


# ---------------------------------------------------------------------------------------------
# The reference's live configuration (survey-default family: free gauge, 2 % outliers, left image
# only).  Most such windows are not reproducible even by the reference under a change of summation
# order (tests/windows.py, DESIGN.md 4.2: the Huber gate's rounding residue, and landmarks that run
# off to ~1e15 along their viewing rays).  These seeds are: the oracle's final chi2 moves < 1e-12
# across OpenMP thread counts, with the reference gate (gate 0) or with the residue taken as 0
# (gate 1, the diagnostic mode on both sides).  On them the full solve is held to the north-star bar.
# ---------------------------------------------------------------------------------------------
DEFAULT_REPRODUCIBLE = [("mini", 2, 0), ("mini", 6, 0), ("C1", 5, 1), ("C1", 6, 1), ("mini", 1, 1), ("mini", 4, 1),
                        ("mini", 11, 1), ("C2", 0, 1), ("C2", 10, 1)]


@pytest.mark.parametrize("cfg,seed,gate", DEFAULT_REPRODUCIBLE)
def test_full_solve_parity_survey_default(cfg, seed, gate):
    w = window(cfg, seed=seed)
    assert w.get("pose_fixed") is None and not np.any(w["obs_cam"])   # gauge free, left image only
    o, spread, its = oracle_envelope(w, threads=(1, 2, 8), gate_mode=gate)
    assert spread < 1e-12, f"oracle not reproducible (spread {spread:.1e})"
    g = lego_ba.Solver(gate_mode=gate).solve(w)
    assert g["iterations"] in its and g["trials"] == o["trials"]
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-6
    if gate == 1:
        assert np.allclose(g["trace_chi2"], o["trace_chi2"], rtol=1e-6)
    else:
        # the reference gate: the final chi2 is reproducible on these seeds, the path to it is not
        # (a Huber-tail edge's weight follows the sign of a rounding residue, base_edge.cpp:55)
        assert rel(g["trace_chi2"][0], o["trace_chi2"][0]) < 1e-12
    # States: the gauge is held only by lambda, and with the reference gate a few weakly held
    # landmarks move by up to ~1e-3 m between the oracle's own summation orders (its final chi2
    # does not).  Gate 1: after the Sim(3) alignment of App. B2 the solutions agree to 1e-6.
    # Gate 0: within 10x the oracle's own state spread.
    if gate == 1:
        lm_err, cam_err, _ = aligned_errors(g["lm_xyz"], o["lm_xyz"], g["pose_Tcw"], o["pose_Tcw"])
        assert lm_err < 1e-6 and cam_err < 1e-6
        assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-5)
    else:
        _, lm_sp, pose_sp = oracle_state_spread(w, threads=(1, 2, 8), gate_mode=gate)
        assert np.abs(g["lm_xyz"] - o["lm_xyz"]).max() <= max(1e-5, 10 * lm_sp)
        assert np.abs(g["pose_Tcw"] - o["pose_Tcw"]).max() <= max(1e-5, 10 * pose_sp)


# ---------------------------------------------------------------------------------------------
# Landmarks with a single edge: rank-2 H_ll.  In the live pipeline every freshly
# triangulated landmark has one usable (left) observation.
# ---------------------------------------------------------------------------------------------
def k1_window(seed, family):
    w = window("mini", seed=seed, family=family, pose_mode=1, k_min=1, k_max=8)
    k = np.bincount(w["obs_lm"], minlength=len(w["lm_xyz"]))
    assert np.sum(k == 1) > 20
    return w, int(np.sum(k == 1))


@pytest.mark.parametrize("seed,family", [(0, "stable_noout"), (1, "default"), (2, "stable")])
def test_single_edge_landmarks_reference_semantics(seed, family):
    """degenerate_guard 0: the reference inverts each rank-2 H_ll with PartialPivLU
    (problem.cpp:396-400).  Some of those inverses are inf, which makes every S entry NaN through
    the dense GEMMs (0 * inf, :402-404); Eigen's LDLT then yields a NaN step (its triangular solves
    run even when the first pivot is invalid), so every candidate keeps its states up to
    VertexPose::add's re-orthonormalisation of a zero update, and every trial is rejected
    (2 iterations x 10 trials).  The solver reproduces that outcome exactly (it poisons the step on
    any single-edge landmark), including the per-edge rho0 "as last evaluated"."""
    w, nk1 = k1_window(seed, family)
    o = ob.solve(w, variant=0)        # the literal dense form: the reference's NaN propagation
    assert np.array_equal(o["edge_robust_chi2"], ob.solve(w)["edge_robust_chi2"])
    assert o["accepted"] == 0 and o["iterations"] == 2 and o["trials"] == 20   # the reference stalls
    g = lego_ba.Solver().solve(w)
    assert g["degenerate"] >= nk1
    assert (g["iterations"], g["trials"], g["accepted"]) == (o["iterations"], o["trials"], o["accepted"])
    assert g["chi2_final"] == g["chi2_initial"] and rel(g["chi2_final"], o["chi2_final"]) < 1e-13
    assert np.array_equal(g["pose_Tcw"], w["pose_Tcw"]) and np.array_equal(g["lm_xyz"], w["lm_xyz"])
    assert np.array_equal(g["edge_robust_chi2"], o["edge_robust_chi2"])


@pytest.mark.parametrize("seed", [0, 3])
def test_single_edge_landmarks_guard(seed):
    """degenerate_guard 1 (opt-in deviation): single-edge landmarks are held fixed (no Schur term, no
    update) and the solve proceeds; the oracle restates the same guard."""
    w, nk1 = k1_window(seed, "stable_noout")
    o, spread, its = oracle_envelope(w, threads=(1, 2, 8), degenerate_guard=1)
    assert spread < 1e-12 and o["accepted"] > 0
    g = lego_ba.Solver(degenerate_guard=1).solve(w)
    assert g["degenerate"] == nk1
    assert g["iterations"] in its and g["trials"] == o["trials"]
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-6
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-6)
    assert np.allclose(g["lm_xyz"], o["lm_xyz"], atol=1e-6)
    k = np.bincount(w["obs_lm"], minlength=len(w["lm_xyz"]))
    assert np.array_equal(g["lm_xyz"][k == 1], w["lm_xyz"][k == 1])   # held fixed
    # one trial at the per-linearisation bar
    g1 = lego_ba.Solver(degenerate_guard=1, max_iters=1, max_trials=1).solve(w)
    o1 = ob.solve(w, degenerate_guard=1, max_iters=1, max_trials=1)
    assert rel(g1["chi2_final"], o1["chi2_final"]) < 1e-9
    assert np.allclose(g1["pose_Tcw"], o1["pose_Tcw"], atol=1e-9)
    assert np.allclose(g1["lm_xyz"], o1["lm_xyz"], atol=1e-7)


# ---------------------------------------------------------------------------------------------
# C4 (BASELINE configs[3]): 20 KF / 500 k landmarks / 4 M observations, the multi-GPU window, here
# on one GPU against the oracle.
# ---------------------------------------------------------------------------------------------
def test_c4_window_one_gpu_parity():
    """C4 at full size.  With the reference Huber gate (base_edge.cpp:55) the C4 trajectory is not
    reproducible even by the oracle: 8 vs 5 OpenMP threads already differ by 2e-5 at iteration 2
    and end after 7 iterations at final chi2 7e-10 apart (a few edges sit in the Huber tail, and
    the gate's rounding residue flips their weights).  With the residue taken as 0 on both sides
    (gate_mode 1) the oracle is reproducible to 1e-14 across thread counts, and the GPU is held to
    the north-star bar on it: same iterations and trials, trace and final chi2, poses, landmarks.
    With the reference gate the GPU must land in the same basin (final chi2 to 1e-5)."""
    w = window("C4", seed=0, family="stable_noout")
    assert len(w["obs_pose"]) == 4_000_000
    g = lego_ba.Solver(gate_mode=1).solve(w)
    o, spread, its = oracle_envelope(w, threads=(8, 16), gate_mode=1)
    assert spread < 1e-12 and its == {o["iterations"]}
    assert g["iterations"] == o["iterations"] and g["trials"] == o["trials"]
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-6
    assert np.allclose(g["trace_chi2"], o["trace_chi2"], rtol=1e-9)
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-6)
    assert np.allclose(g["lm_xyz"], o["lm_xyz"], atol=1e-6)
    assert np.all(np.diff(g["trace_chi2"]) <= 0)
    g0 = lego_ba.Solver().solve(w)
    o0 = ob.solve(w, n_threads=16)
    assert g0["chi2_final"] < g0["chi2_initial"] and rel(g0["chi2_initial"], o0["chi2_initial"]) < 1e-12
    assert rel(g0["chi2_final"], o0["chi2_final"]) < 1e-5


# ---------------------------------------------------------------------------------------------
# The per-trial exchange must issue the same number of collectives on every rank: the stop trial is
# decided by identical all-reduced data, and each rank tops up to min(stop trial + depth, cap).
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("depth,cfg,family,batch", [(1, "C2", "stable_noout", True), (2, "C2", "stable_noout", True),
                                                     (5, "C2", "stable_noout", True), (2, "mini", "default", False),
                                                     (2, "mini", "default", True)])
def test_collective_count_is_a_function_of_the_stop_trial(monkeypatch, depth, cfg, family, batch):
    """(mini, default: rejections followed by acceptances, so re-linearisation chains -- or, batched, retrials --
    run through the exchange and the controller's own decision, the path every sharded solve takes)"""
    monkeypatch.setenv("LH_FORCE_RCCL", "1")
    if not batch:   # one trial per chain: the re-linearisation chains counted below
        monkeypatch.setenv("LH_NO_BATCH", "1")
    w = window(cfg, seed=0, family=family)
    s = lego_ba.Solver(trials_per_sync=depth)
    counts = set()
    for _ in range(3):
        r = s.solve(w)
        counts.add(s.comm_count())
    # chains: the trials, plus a re-linearisation per evaluate-only acceptance (at most one per iteration), less the
    # rungs a batch decided beyond its first (at most 15 per batch)
    assert counts == {1 + min(s.chains() + depth, 10 * (10 + 1))} and s.chains() + 15 * s.batch()[1] >= r["trials"]
    if family == "default":
        assert s.chains() > r["trials"] if not batch else (s.batch()[1] > 0 and s.chains() < r["trials"])
        monkeypatch.setenv("LH_NO_EVAL_FIRST", "1")
        monkeypatch.setenv("LH_NO_BATCH", "1")
        t = lego_ba.Solver(trials_per_sync=depth)
        f = t.solve(w)
        t.close()
        for k in ("iterations", "trials", "chi2_final", "lambda_final"):
            assert f[k] == r[k], k
        for k in ("pose_Tcw", "lm_xyz", "edge_robust_chi2"):
            assert np.array_equal(f[k], r[k]), k
    s.close()


# A trial of the final LM iteration only evaluates the candidate (ctrl.evo): its linearisation could
# never be used.  LH_NO_EVO=1 (read when a window is uploaded) linearises every trial in full; both
# runs must agree bit for bit, including runs that reject in the final iteration.
@pytest.mark.parametrize("cfg,family,kw", [
    ("C2", "stable", {}),
    ("C2", "default", {}),
    ("C1", "default", dict(max_iters=3, max_trials=3)),
    ("C2", "default", dict(strategy=1, max_iters=4)),
    ("C1", "stable", dict(max_iters=1, max_trials=1)),
    ("W24s", "stable_noout", dict(max_iters=3)),
])
def test_final_iteration_trials_evaluate_only(cfg, family, kw, monkeypatch):
    w = window(cfg, seed=4, family=family)
    monkeypatch.setenv("LH_NO_EVO", "1")
    s = lego_ba.Solver(**kw)
    full = s.solve(w)
    s.close()
    monkeypatch.delenv("LH_NO_EVO")
    s = lego_ba.Solver(**kw)
    evo = s.solve(w)
    s.close()
    for k in ("iterations", "trials", "accepted", "chi2_final", "lambda_final"):
        assert full[k] == evo[k], k
    for k in ("pose_Tcw", "lm_xyz", "edge_robust_chi2", "trace_chi2", "trace_lambda"):
        assert np.array_equal(full[k], evo[k]), k


# After a rejection a trial only evaluates (prm.eval_first): a run of rejections (every solve that stops on a
# stalled chi2 ends with max_trials of them, problem.cpp:189-218) pays evaluations only, and an acceptance
# among them costs one re-linearisation chain (ctrl.relin).  LH_NO_EVAL_FIRST=1 linearises every trial
# outside the final iteration; both must agree bit for bit on every controller, and the windows below
# (rejections followed by acceptances) must run re-linearisation chains past their trials.  Most are chaotic
# windows, picked on the current kernels' trajectories (`scripts/eval_first_cases.py` lists the chains per
# window): a change of rounding in k_lin moves where their rejections fall, and the list with it.
EVAL_FIRST_CASES = [
    ("C1 k_ctrl", dict(cfg="C1", seed=0), {}, "k_ctrl"),
    ("mini k_ctrl", dict(cfg="mini", seed=0), {}, "k_ctrl"),
    ("C2 strategy 1", dict(cfg="C2", seed=0), dict(strategy=1), "k_ctrl"),
    ("C2 PCG", dict(cfg="C2", seed=0), dict(linear_solver=lego_ba.LH_SOLVER_PCG), "k_ctrl"),
    ("C2 max_trials 3", dict(cfg="C2", seed=3), dict(max_trials=3), "k_ctrl"),
    ("P32 dense", dict(P=32, L=3000, seed=1, pose_mode=1, k_min=2, k_max=8), {}, "k_ctrl_g"),
    ("P96 banded", dict(P=96, L=6000, seed=2), {}, "k_ctrl_b"),
    ("P96 PCG", dict(P=96, L=6000, seed=2), dict(linear_solver=lego_ba.LH_SOLVER_PCG), "k_ctrl_p"),
    ("C2 fp32 Jacobians", dict(cfg="C2", seed=0), dict(precision=lego_ba.LH_PREC_FP32_RESID), "k_ctrl"),
    ("mini 4 cameras", dict(cfg="mini", seed=1, cams=4), {}, "k_ctrl"),
]


def _eval_first_run(wargs, kw, env_off, monkeypatch):
    from windows import multi_camera
    wargs = dict(wargs)
    cams = wargs.pop("cams", 0)
    w = window(wargs.pop("cfg"), seed=wargs.pop("seed")) if "cfg" in wargs else \
        lego_ba.generate_window(k=8, **wargs)
    if cams:
        w = multi_camera(w, cams, seed=1)
    if env_off:
        monkeypatch.setenv("LH_NO_EVAL_FIRST", "1")
    s = lego_ba.Solver(**kw)
    r = s.solve(w)
    r["controller"] = s.controller()
    r["chains"] = s.chains()
    r["ladder"] = s.ladder()
    s.close()
    monkeypatch.delenv("LH_NO_EVAL_FIRST", raising=False)
    return r


def test_trials_after_a_rejection_evaluate_first(monkeypatch):
    monkeypatch.setenv("LH_NO_BATCH", "1")   # one trial per chain: the chain counts below (batches: the test after)
    for name, wargs, kw, ctrl in EVAL_FIRST_CASES:
        full = _eval_first_run(wargs, kw, True, monkeypatch)
        ef = _eval_first_run(wargs, kw, False, monkeypatch)
        assert ef["controller"] == ctrl, name
        for k in ("iterations", "trials", "accepted", "chi2_final", "lambda_final", "chi2_initial"):
            assert full[k] == ef[k], (name, k)
        for k in ("pose_Tcw", "lm_xyz", "edge_robust_chi2", "trace_chi2", "trace_lambda"):
            assert np.array_equal(full[k], ef[k]), (name, k)
        assert full["chains"] == full["trials"] and ef["chains"] >= ef["trials"], name


# The re-linearisation chain on windows that must take it (tests/windows.py RELIN_WINDOWS: a rejection and then
# an acceptance inside an iteration before the last, by a margin no summation order moves; the oracle's
# accept/reject string is pinned by scripts/relin_windows.py).  The GPU must take the oracle's decisions (same
# iterations, trials, acceptances), run more chains than trials, and equal the eval-first-off solve bit for bit.
def _relin_run(gen, opt, env, monkeypatch):
    from windows import relin_window
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    s = lego_ba.Solver(max_iters=3, **opt)
    r = s.solve(relin_window(gen))
    r["controller"], r["chains"], r["ladder"] = s.controller(), s.chains(), s.ladder()
    s.close()
    for k in env:
        monkeypatch.delenv(k)
    return r


@pytest.mark.parametrize("case", range(9))
def test_rejection_then_acceptance_relinearises(case, monkeypatch):
    from windows import RELIN_WINDOWS, relin_window
    kind, gen, opt, dec, ctrl = RELIN_WINDOWS[case]
    monkeypatch.setenv("LH_NO_BATCH", "1")   # one trial per chain: the chain counts below (batches: test below)
    o = ob.solve(relin_window(gen), max_iters=3, **opt)
    assert (o["iterations"], o["trials"], o["accepted"]) == (3, len(dec), dec.count("A")), kind
    ef = _relin_run(gen, opt, {}, monkeypatch)
    full = _relin_run(gen, opt, {"LH_NO_EVAL_FIRST": "1"}, monkeypatch)
    assert ef["controller"] == ctrl, kind
    assert (ef["iterations"], ef["trials"], ef["accepted"]) == (o["iterations"], o["trials"], o["accepted"]), kind
    assert ef["chains"] > ef["trials"] and full["chains"] == full["trials"], (kind, ef["chains"], ef["trials"])
    for k in ("iterations", "trials", "accepted", "chi2_final", "lambda_final", "chi2_initial", "pcg_iterations"):
        assert full[k] == ef[k], (kind, k)
    for k in ("pose_Tcw", "lm_xyz", "edge_robust_chi2", "trace_chi2", "trace_lambda"):
        assert np.array_equal(full[k], ef[k]), (kind, k)
    assert ef["chi2_final"] < ef["chi2_initial"]
    # the lambda ladder on the same window: bitwise the one-rung run, and every rejection with a built rung used it
    # (with the ladder off none does)
    one = _relin_run(gen, opt, {"LH_NO_LADDER": "1"}, monkeypatch)
    for k in ("iterations", "trials", "accepted", "chi2_final", "lambda_final", "pcg_iterations"):
        assert one[k] == ef[k], (kind, k)
    for k in ("pose_Tcw", "lm_xyz", "edge_robust_chi2", "trace_chi2", "trace_lambda"):
        assert np.array_equal(one[k], ef[k]), (kind, k)
    assert one["ladder"] == (1, 0), kind
    assert ef["ladder"] == (10, _ladder_skips(dec, 10, eager=True)), (kind, ef["ladder"])
    lazy = _relin_run(gen, opt, {"LH_LADDER_LAZY": "1"}, monkeypatch)
    assert lazy["ladder"] == (10, _ladder_skips(dec, 10, eager=False)), (kind, lazy["ladder"])
    assert lazy["chi2_final"] == ef["chi2_final"] and np.array_equal(lazy["pose_Tcw"], ef["pose_Tcw"]), kind


def _ladder_skips(dec, rungs, eager):
    """The rejections of a decision string that land on a built rung.  The initial linearisation's controller builds
    no ladder; a later factor builds `rungs` (eager: every one, each acceptance's; lazy: only the first rejection of
    a run that found no rung).  The last decision stops the loop and needs no step."""
    lad, lad_n, n = 0, 1, 0
    for i, d in enumerate(dec):
        last = i == len(dec) - 1
        if d == "A":
            lad, lad_n = 0, (rungs if eager else 1)
        elif lad + 1 < lad_n and not last:
            lad, n = lad + 1, n + 1
        else:
            lad, lad_n = 0, rungs
    return n


# The lambda ladder: a controller that factors (LH_LADDER_LAZY=1: only one that factors after a
# rejection) also factors the same system at the lambdas the next rejections would set
# (problem.cpp:550-551, STRATEGY1 :576), one workgroup per rung, and a rejection onto a built rung skips its
# factor.  Every rung runs the serial controller's code at bit-identical lambdas, so the solve must equal the
# one-rung run (LH_NO_LADDER=1) bit for bit on every controller (k_ctrl LDL^T and PCG, k_ctrl_b, k_ctrl_g,
# k_ctrl_p: the last two, and the initial linearisation's controller, take the decision themselves and publish it
# to their rung workgroups), and the windows with rejection runs must have used rungs.
def _ladder_run(wargs, kw, env, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    r = _eval_first_run(wargs, kw, False, monkeypatch)
    for k in env:
        monkeypatch.delenv(k)
    return r


@pytest.mark.parametrize("eager", [False, True])
def test_lambda_ladder_is_bitwise_the_serial_chain(monkeypatch, eager):
    used = []
    for name, wargs, kw, ctrl in EVAL_FIRST_CASES:
        env = {} if eager else {"LH_LADDER_LAZY": "1"}
        serial = _ladder_run(wargs, kw, {"LH_NO_LADDER": "1"}, monkeypatch)
        lad = _ladder_run(wargs, kw, env, monkeypatch)
        assert serial["ladder"] == (1, 0), name
        for k in ("iterations", "trials", "accepted", "chi2_final", "lambda_final", "chi2_initial", "pcg_iterations"):
            assert serial[k] == lad[k], (name, k)
        for k in ("pose_Tcw", "lm_xyz", "edge_robust_chi2", "trace_chi2", "trace_lambda"):
            assert np.array_equal(serial[k], lad[k]), (name, k)
        rungs, skipped = lad["ladder"]
        assert rungs == min(kw.get("max_trials", 10), 16), name
        if skipped > 0:
            used.append((name, ctrl))
        assert skipped <= lad["trials"] - lad["accepted"], name
    assert len(used) >= 4, used


# Batched rejection runs: after a rejection onto a built rung, one chain evaluates the rungs up
# to the last built one (or the iteration's last trial) and k_reduce decides them in order; an acceptance among them
# is re-run by the next chain as a full trial at that rung (lh_ctrl.retrial), whose decision commits it.  Every
# rung is evaluated at its own step and lambda with the serial evaluate-only path's arithmetic and summation order,
# so the solve must equal the one-rung-per-chain run (LH_NO_BATCH=1) bit for bit: the LM counts and trace, the
# states, the per-edge rho0 "as last evaluated" (a rung buffer when the solve stops inside a batch) and the device
# outlier pass on it; and the windows with rejection runs must have run batches (fewer chains).
def _batch_run(w, kw, env, monkeypatch, th):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    s = lego_ba.Solver(**kw)
    r = s.solve(w)
    r["chains"], r["batch"], r["retrials"] = s.chains(), s.batch(), s.batch_detail()[2]
    o = s.solve(w, outlier_chi2_th=th)
    r["is_outlier"], r["n_outlier"] = o["is_outlier"].copy(), o["n_outlier"]
    s.close()
    for k in env:
        monkeypatch.delenv(k)
    return r


def _batch_windows():
    from windows import RELIN_WINDOWS, relin_window, multi_camera
    out = []
    for name, wargs, kw, ctrl in EVAL_FIRST_CASES:
        wa = dict(wargs)
        cams = wa.pop("cams", 0)
        w = window(wa.pop("cfg"), seed=wa.pop("seed")) if "cfg" in wa else lego_ba.generate_window(k=8, **wa)
        if cams:
            w = multi_camera(w, cams, seed=1)
        out.append((name, w, kw, ctrl))
    for kind, gen, opt, dec, ctrl in RELIN_WINDOWS:
        out.append(("relin " + kind, relin_window(gen), dict(max_iters=3, **opt), ctrl))
    # the bench's live configuration (a stalled solve ends every run of it with max_trials rejections)
    out.append(("C3 live", window("C3", seed=0, family="default"), {}, "k_ctrl"))
    # sixteen rungs (the most, LH_LAD): batches past k_reduce's ten rungs per round of loads
    out.append(("C3 live 16 trials", window("C3", seed=0, family="default"), dict(max_trials=16), "k_ctrl"))
    return out


@pytest.mark.parametrize("env", [{}, {"LH_BATCH_MAX": "3"}, {"LH_LADDER_LAZY": "1"}])
def test_batched_rejection_runs_are_bitwise_the_serial_chain(monkeypatch, env):
    batched, retrials = [], [0, 0]
    for name, w, kw, ctrl in _batch_windows():
        th = 5.991
        serial = _batch_run(w, kw, dict(env, LH_NO_BATCH="1"), monkeypatch, th)
        bat = _batch_run(w, kw, env, monkeypatch, th)
        assert serial["batch"][0] == 1, name
        for k in ("iterations", "trials", "accepted", "chi2_final", "lambda_final", "chi2_initial", "pcg_iterations",
                  "n_outlier"):
            assert serial[k] == bat[k], (name, k)
        for k in ("pose_Tcw", "lm_xyz", "edge_robust_chi2", "trace_chi2", "trace_lambda", "is_outlier"):
            assert np.array_equal(serial[k], bat[k]), (name, k)
        bmax, nb = bat["batch"]   # every controller (k_reduce decides with k_ctrl and k_ctrl_b, else the controller)
        assert bmax == min(kw.get("max_trials", 10), int(env.get("LH_BATCH_MAX", 16))), name
        # a batch replaces its rungs' chains by one, plus the retrial of an acceptance that stopped the loop (where
        # the serial run's accepted evaluate-only trial was its last chain)
        if nb > 0:
            batched.append(name)
            retrials[0] += bat["retrials"][0]
            retrials[1] += bat["retrials"][1]
            assert bat["chains"] <= serial["chains"] + nb, (name, bat["chains"], serial["chains"], nb)
        else:
            assert bat["chains"] == serial["chains"], name
        if name == "C3 live":
            assert bat["chains"] < serial["chains"], (bat["chains"], serial["chains"])
    assert "C3 live" in batched and len(batched) >= 10, batched
    # both kinds of acceptance inside a batch ran: re-run as a full trial, and re-run as the stopping trial
    if not env:
        assert retrials[0] > 0 and retrials[1] > 0, retrials


# ---------------------------------------------------------------------------------------------
# Camera rigs of 3 and 4 cameras with non-identity extrinsic rotations (EdgeProjection takes any
# Camera::pose_, lego_types.h:211-215, 229-253; the ABI allows 4 cameras).  Landmarks seen by up to
# 16 poses through 4 cameras give k_lin<6> its largest LDS image (T = 6 with 4 cameras' pose tables).
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n_cams,kmin,kmax,mode", [(3, 8, 8, 0), (4, 8, 8, 0), (4, 2, 10, 1), (4, 11, 16, 1)])
def test_multi_camera_rigs_with_rotated_extrinsics(n_cams, kmin, kmax, mode):
    from windows import STABLE, multi_camera
    w = lego_ba.generate_window(P=20, L=3000, k=kmin, k_max=kmax, seed=7, pose_mode=mode,
                                **dict(STABLE, outlier_frac=0.0))
    f = np.zeros(20, np.uint8)
    f[0] = 1
    w["pose_fixed"] = f
    w = multi_camera(w, n_cams, seed=7)
    assert set(np.unique(w["obs_cam"])) == set(range(n_cams))
    # residual, robust weight and rho0 through the rotated extrinsics: bitwise the oracle's
    g0 = lego_ba.Solver(max_iters=0).solve(w)
    o0 = ob.solve(w, max_iters=0)
    assert np.array_equal(g0["edge_robust_chi2"], o0["edge_robust_chi2"])
    g = lego_ba.Solver(max_iters=1, max_trials=1).solve(w)
    o = ob.solve(w, max_iters=1, max_trials=1)
    assert rel(g["chi2_final"], o["chi2_final"]) < 1e-9
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-9)
    assert np.allclose(g["lm_xyz"], o["lm_xyz"], atol=1e-7)
    gf = lego_ba.Solver().solve(w)
    of, spread, its = oracle_envelope(w, threads=(1, 2, 8))
    assert gf["iterations"] in its
    assert rel(gf["chi2_final"], of["chi2_final"]) < max(1e-6, 10 * spread)
    assert gf["chi2_final"] < gf["chi2_initial"]


def test_five_cameras_are_unsupported():
    from windows import STABLE, multi_camera
    w = multi_camera(lego_ba.generate_window(P=10, L=300, k=8, seed=1, **STABLE), 4, seed=1)
    w["cam_ext"] = np.vstack([w["cam_ext"], w["cam_ext"][:1]])
    w["obs_cam"] = w["obs_cam"].copy()
    w["obs_cam"][:5] = 4
    with pytest.raises(lego_ba.LhError) as e:
        lego_ba.Solver().solve(w)
    assert e.value.status == lego_ba.LH_E_UNSUPPORTED


@pytest.mark.parametrize("cfg,seed,family", [("C3", 0, "stable_noout"), ("C3", 1, "stable_noout")])
def test_two_chain_schedule_matches_the_one_chain_solve(monkeypatch, cfg, seed, family):
    """k_ctrl's two-chain LDL^T (opt-in LH_ND=1, lh_ctrl_nd_plan) on windows that split (C3: A = 4, S = 8,
    B = 8 poses): a different elimination order, so the same LM path and the final chi2 to rounding."""
    w = window(cfg, seed=seed, family=family)
    s0 = lego_ba.Solver()
    a = s0.solve(w)
    s0.close()
    monkeypatch.setenv("LH_ND", "1")
    s1 = lego_ba.Solver()
    b = s1.solve(w)
    assert s1.controller() == "k_ctrl"
    s1.close()
    assert (b["iterations"], b["trials"]) == (a["iterations"], a["trials"])
    assert rel(b["chi2_final"], a["chi2_final"]) <= 1e-9
    assert np.allclose(b["pose_Tcw"], a["pose_Tcw"], atol=1e-7)

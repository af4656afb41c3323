"""CPU tests of the controllers' per-step work units (lh_common.h lh_ctrl_units).

k_ctrl and k_ctrl_b factor the reduced system S + lambda D in natural pose order by a blocked
right-looking LDL^T (8-column blocks); per step, the host-built table deals the trailing 16x16 tiles
of the tile rows the envelope of S reaches to the unit waves.  Here the table is replayed in numpy
at tile granularity with the kernels' operand algebra (L_I = a_I N, T_I = L_I (N Delta)^T,
A_IJ -= T_I a_J^T, the rhs riding along, z = b N, x = L^-T z by blocks), and the solution is held
against numpy's solve: a tile the table forgets, doubles, or assigns past the window shows up as a
wrong x.  The banded table (k_ctrl_b) is also checked against its streaming window: every tile a step
touches has been loaded into the 8-tile-row circular window (tile row I enters at step 2I - 14)."""
import numpy as np
import pytest

import lego_ba

VALID, STORE = 0x8000, 0x4000


def envelope_fcb(n, pose_first):
    """First 8-column block each 16-row tile row reaches (lh_host.cpp): row r of pose p starts at 6 f(p)."""
    NE = (n + 15) & ~15
    fc = np.array([6 * pose_first[r // 6] if r < n else r for r in range(NE)])
    return (fc.reshape(-1, 16).min(axis=1) >> 3).astype(np.int32)


def banded_system(P, span, rng):
    """S + lambda I of a window whose landmarks couple poses at most `span` apart (SPD)."""
    n = 6 * P
    B = np.zeros((n, n))
    for p in range(P):
        for q in range(p, min(P, p + span + 1)):
            B[6 * p:6 * p + 6, 6 * q:6 * q + 6] = rng.standard_normal((6, 6))
    S = B @ B.T   # couples poses up to `span` apart on each side... keep only the band
    for p in range(P):
        for q in range(P):
            if abs(p - q) > span:
                S[6 * p:6 * p + 6, 6 * q:6 * q + 6] = 0.0
    S = S + np.diag(np.abs(S).sum(axis=1) + 10.0 ** rng.uniform(0, 3, n))   # diagonally dominant: SPD
    pose_first = [max(0, p - span) for p in range(P)]
    return S, pose_first


def replay(S, b, units, steps, band=False):
    """The kernels' blocked LDL^T + solve, driven by the unit table; returns x."""
    n = len(b)
    NE, nb = (n + 15) & ~15, (n + 7) & ~7
    A = np.eye(NE)
    A[:n, :n] = S
    rhs = np.zeros(NE)
    rhs[:n] = b
    A = np.tril(A)
    L = np.zeros((NE, NE))
    NDs, Ns, Ds = [], [], []

    def factor(k0):   # 8x8 LDL^T of A[k0:k0+8, k0:k0+8] (lower part)
        M = np.tril(A[k0:k0 + 8, k0:k0 + 8])
        M = M + np.tril(M, -1).T
        Lb, D = np.eye(8), np.zeros(8)
        W = M.copy()
        for q in range(8):
            D[q] = W[q, q]
            dl = D[q] if D[q] != 0 else 1.0
            Lb[q + 1:, q] = W[q + 1:, q] / dl
            W[q + 1:, q + 1:] -= np.outer(Lb[q + 1:, q], W[q, q + 1:])
        dl = np.where(D != 0, D, 1.0)
        N = np.linalg.inv(np.diag(dl) @ Lb.T)   # (Delta L^T)^-1
        A[k0:k0 + 8, k0:k0 + 8] = np.diag(D) + np.tril(Lb, -1) * 0   # D on the diagonal
        return N, N @ np.diag(dl), D

    def tile_row(k0, rb, jb0, jb1, store, N, ND):
        m0 = k0 + 8
        a = A[rb:rb + 16, k0:k0 + 8].copy()
        a[np.arange(rb, rb + 16) < m0] = 0.0          # the block's own rows are masked
        Li = a @ N
        Ti = Li @ ND.T
        if store:
            rows = np.arange(rb, rb + 16)
            keep = rows >= m0
            L[rows[keep], k0:k0 + 8] = Li[keep]
            rhs[rows[keep]] -= Ti[keep] @ rhs[k0:k0 + 8]
        for cb in range(jb0, jb1, 16):
            aj = A[cb:cb + 16, k0:k0 + 8]
            upd = Ti @ aj.T
            for i in range(16):
                for j in range(16):
                    r, c = rb + i, cb + j
                    if r >= m0 and c >= m0 and c <= r:
                        A[r, c] -= upd[i, j]

    N, ND, D = factor(0)
    Ns.append(N); NDs.append(ND); Ds.append(D)
    z = np.zeros(NE)
    for t in range(nb // 8):
        k0, m0 = 8 * t, 8 * t + 8
        N, ND = Ns[t], NDs[t]
        zz = rhs[k0:k0 + 8] @ N
        z[k0:k0 + 8] = np.where(np.abs(Ds[t]) > 2.2250738585072014e-308, zz, 0.0)
        if m0 >= nb:
            continue
        g0 = m0 >> 4
        pending = []   # every unit reads the operands as they were before the step
        if units[0, t] & VALID:
            pending.append((16 * g0, 16 * g0, 16 * g0 + 16, False))
        for w in range(1, 16):
            u = int(units[w, t])
            if not u & VALID:
                continue
            I, jb0, jb1 = g0 + (u & 7), g0 + ((u >> 3) & 7), g0 + ((u >> 6) & 15)
            pending.append((16 * I, 16 * jb0, 16 * jb1, bool(u & STORE)))
        snapshot = A.copy()
        for rb, j0, j1, st in pending:
            saved = A
            A = snapshot.copy()
            before = A.copy()
            tile_row(k0, rb, j0, j1, st, N, ND)
            delta = A - before
            A = saved
            A += delta
        Nn, NDn, Dn = factor(m0)
        Ns.append(Nn); NDs.append(NDn); Ds.append(Dn)
    # x = L^-T z by blocks: x_b = ND_b y_b, then y_r -= sum L[b][r] x_b
    y = z.copy()
    for KB in range(nb - 8, -1, -8):
        xb = NDs[KB // 8] @ y[KB:KB + 8]
        y[:KB] -= L[KB:KB + 8, :KB].T @ xb
        y[KB:KB + 8] = xb
    return y[:n]


@pytest.mark.parametrize("P,span,seed", [(20, 7, 0), (21, 20, 1), (20, 3, 2), (13, 12, 3), (17, 5, 4)])
def test_k_ctrl_units_solve(P, span, seed):
    rng = np.random.default_rng(seed)
    S, pf = banded_system(P, span, rng)
    n = 6 * P
    fcb = np.zeros(8, np.int32)
    e = envelope_fcb(n, pf)
    fcb[:len(e)] = e
    units, worst = lego_ba.ctrl_units(n, fcb)
    assert worst <= 15
    b = rng.standard_normal(n)
    x = replay(S, b, units, 16)
    xr = np.linalg.solve(S, b)
    assert np.linalg.norm(x - xr) <= 1e-10 * np.linalg.norm(xr)


def test_k_ctrl_units_dense_envelope_matches_the_round_3_split():
    """A dense envelope (sharded solves, the probe): every tile row active, half tile rows per unit."""
    units, worst = lego_ba.ctrl_units(120, np.zeros(8, np.int32))
    assert worst == 15
    assert all(units[w, 0] & VALID for w in range(16))   # step 0: wave 0 and all 15 unit waves


@pytest.mark.parametrize("P,span,seed", [(22, 7, 0), (40, 7, 1), (64, 10, 2), (96, 7, 3), (30, 14, 4), (30, 20, 5),
                                         (96, 15, 6)])
def test_k_ctrl_b_units_solve_and_window(P, span, seed):
    rng = np.random.default_rng(seed)
    S, pf = banded_system(P, span, rng)
    n = 6 * P
    NE = (n + 15) & ~15
    fcb = envelope_fcb(n, pf)
    units, worst = lego_ba.ctrl_units(n, fcb, band=True)
    banded = all(fcb[I] >= 2 * I - 13 for I in range(8, NE // 16)) and worst <= 15
    if span <= 15:
        assert banded       # sliding-window bands (the reference window is 15 keyframes, map.h:82)
    if not banded:
        return
    # the stream loaders (waves 12-15) take units only in steps that need more than the 11 unit waves
    for t in range(units.shape[1]):
        if np.any(units[12:, t] & VALID):
            assert int(np.count_nonzero(units[1:, t] & VALID)) > 11
    # every tile a step touches is inside the window and already loaded
    for t in range(units.shape[1]):
        g0 = (8 * t + 8) >> 4
        glo = t // 2
        for w in range(16):
            u = int(units[w, t])
            if not u & VALID:
                continue
            j0, j1 = (u >> 3) & 7, (u >> 6) & 15
            rows = [g0] if w == 0 else [g0 + (u & 7)] + ([g0 + j0, g0 + j1 - 1] if j1 > j0 else [])
            for I in rows:
                assert glo <= I <= glo + 7
                assert I < 8 or t >= 2 * I - 13
    b = rng.standard_normal(n)
    x = replay(S, b, units, units.shape[1], band=True)
    xr = np.linalg.solve(S, b)
    assert np.linalg.norm(x - xr) <= 1e-10 * np.linalg.norm(xr)


# ---- the two-chain schedule (lh_ctrl_nd_plan): k_ctrl's LDL^T as two concurrent chains ----
SRC0, STORE0 = 0x0400, 0x1000


def replay_nd(S, b, nd, debug=False):
    """k_ctrl's two-chain LDL^T (lds_ldlt_solve_nd) driven by the plan's unit words, at tile granularity with
    the kernel's operand algebra (every unit reads the operands as they were before the step); returns x
    in natural order."""
    n = len(b)
    P = n // 6
    NE, nb = (n + 15) & ~15, (n + 7) & ~7
    pos = nd["pos"]
    fr = np.array([6 * pos[r // 6] + r % 6 for r in range(n)])   # natural row -> factor row
    Sp = np.zeros((n, n))
    Sp[np.ix_(fr, fr)] = S
    A = np.eye(NE)
    A[:n, :n] = np.tril(Sp)
    rhs = np.zeros(NE)
    rhs[fr] = b
    L = np.zeros((NE, NE))
    a, sep, lf, T = nd["a"], nd["s"], nd["long_first"], nd["nsteps"]
    bb = P - a - sep
    nl_blk, ns_blk = 6 * (a if lf else bb) // 8, 6 * (bb if lf else a) // 8
    c0 = lambda t: t if t < nl_blk else t + ns_blk          # noqa: E731
    c1 = lambda t: nl_blk + t if t < ns_blk else -1         # noqa: E731
    fac = {}

    def factor(k):
        k0 = 8 * k
        M = np.tril(A[k0:k0 + 8, k0:k0 + 8])
        M = M + np.tril(M, -1).T
        Lb, D, W = np.eye(8), np.zeros(8), M.copy()
        for q in range(8):
            D[q] = W[q, q]
            dl = D[q] if D[q] != 0 else 1.0
            Lb[q + 1:, q] = W[q + 1:, q] / dl
            W[q + 1:, q + 1:] -= np.outer(Lb[q + 1:, q], W[q, q + 1:])
        dl = np.where(D != 0, D, 1.0)
        N = np.linalg.inv(np.diag(dl) @ Lb.T)
        fac[k] = (N, N @ np.diag(dl), D)

    def unit(A, rhs, srcs, smask, stmask, rb, jb0, jb1):
        Ts, mm, ru = {}, 1 << 20, np.zeros(16)
        rows = np.arange(rb, rb + 16)
        for q in (0, 1):
            if not ((smask | stmask) >> q) & 1:   # a stored source need not reach the unit's tiles
                continue
            k = srcs[q]
            k0, m0 = 8 * k, 8 * k + 8
            mm = min(mm, m0)
            N, ND, _ = fac[k]
            Li = A[rb:rb + 16, k0:k0 + 8] @ N
            Ti = Li @ ND.T
            Ti[rows < m0] = 0.0
            Ts[q] = Ti
            if (stmask >> q) & 1:
                keep = rows >= m0
                L[rows[keep], k0:k0 + 8] = Li[keep]
                ru += Ti @ rhs[k0:k0 + 8]
        if stmask:
            keep = rows >= mm
            rhs[rows[keep]] -= ru[keep]
        for cb in range(jb0, jb1, 16):
            acc = np.zeros((16, 16))
            cols = np.arange(cb, cb + 16)
            for q, Ti in Ts.items():
                if not (smask >> q) & 1:
                    continue
                k0 = 8 * srcs[q]
                aj = A[cb:cb + 16, k0:k0 + 8].copy()
                aj[cols < k0 + 8] = 0.0
                acc += Ti @ aj.T
            for i in range(16):
                for j in range(16):
                    r, c = rb + i, cb + j
                    if r >= mm and c >= mm and c <= r:
                        A[r, c] -= acc[i, j]

    factor(c0(0))
    if ns_blk > 0:
        factor(c1(0))
    z = np.zeros(NE)
    units = nd["units"]
    touched = []
    for t in range(T):
        srcs = (c0(t), c1(t))
        for k in srcs:
            if k >= 0:
                k0 = 8 * k
                zz = rhs[k0:k0 + 8] @ fac[k][0]
                z[k0:k0 + 8] = np.where(np.abs(fac[k][2]) > 2.2250738585072014e-308, zz, 0.0)
        pend = []
        for w in range(16):
            u = int(units[w, t])
            if not u & VALID:
                continue
            I = u & 7
            sm, st = (u >> 10) & 3, (u >> 12) & 3
            if w < 2:
                pend.append((sm, 0, 16 * I, 16 * I, 16 * I + 16))
            else:
                pend.append((sm, st, 16 * I, 16 * ((u >> 3) & 7), 16 * ((u >> 6) & 15)))
        owned, rhs_rows = set(), set()   # each tile and each rhs tile row has one owner per step
        for sm, st, rb, j0, j1 in pend:
            for cb in range(j0, j1, 16):
                assert (rb, cb) not in owned
                owned.add((rb, cb))
            if st:
                assert rb not in rhs_rows
                rhs_rows.add(rb)
        snapA, snapR = A.copy(), rhs.copy()
        dA, dR = np.zeros_like(A), np.zeros_like(rhs)
        cells = set()
        for sm, st, rb, j0, j1 in pend:
            A2, R2 = snapA.copy(), snapR.copy()
            unit(A2, R2, srcs, sm, st, rb, j0, j1)
            ch = np.argwhere(A2 != snapA)
            for r, c in ch:            # no two units of a step write one entry
                assert (r, c) not in cells
                cells.add((r, c))
            dA += A2 - snapA
            dR += R2 - snapR
        A, rhs = snapA + dA, snapR + dR
        touched.append(len(pend))
        if t + 1 < T:
            factor(c0(t + 1))
        if srcs[1] >= 0 and c1(t + 1) >= 0:
            factor(c1(t + 1))
    assert len(fac) == nb // 8   # every block factored once
    y = z.copy()
    for KB in range(nb - 8, -1, -8):
        xb = fac[KB // 8][1] @ y[KB:KB + 8]
        y[:KB] -= L[KB:KB + 8, :KB].T @ xb
        y[KB:KB + 8] = xb
    if debug:
        return y[fr], L, fac, z
    return y[fr]


@pytest.mark.parametrize("P,span,seed", [(20, 7, 0), (20, 5, 1), (21, 7, 2), (21, 3, 3), (20, 3, 4), (18, 4, 5)])
def test_k_ctrl_two_chain_schedule_solves(P, span, seed):
    rng = np.random.default_rng(seed)
    S, pf = banded_system(P, span, rng)
    nd = lego_ba.ctrl_nd(pf)
    NB = (6 * P + 7) // 8
    if nd["nsteps"] == 0:
        pytest.skip("no split for this window")
    assert nd["nsteps"] < NB - 1
    assert sorted(nd["pos"]) == list(range(P))
    b = rng.standard_normal(6 * P)
    x = replay_nd(S, b, nd)
    xr = np.linalg.solve(S, b)
    assert np.linalg.norm(x - xr) <= 1e-10 * np.linalg.norm(xr)


def test_k_ctrl_two_chain_schedule_on_c3():
    """C3's window (20 keyframes, chunk windows of 8 consecutive poses): 12 steps instead of 15."""
    pf = [max(0, p - 7) for p in range(20)]
    nd = lego_ba.ctrl_nd(pf)
    assert nd["nsteps"] == 12
    # a separator wide enough to decouple the two parts: no pose past it reaches the part before it
    a, s = nd["a"], nd["s"]
    assert all(pf[q] >= a for q in range(a + s, 20))

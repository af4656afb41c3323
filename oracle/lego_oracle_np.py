"""
lego_oracle_np — TEST INFRASTRUCTURE ONLY.  An independent NumPy restatement
of the reference LEGO-SLAM backend solve (lego::Problem in SLAM mode, driven by
Backend::Optimize), written from the reference source separately from the C
restatement (oracle/lego_oracle.c) so that each checks the other.

PARITY UNPINNED: the reference cannot be compiled here (Eigen3, Sophus, OpenCV
and glog are absent) and it ships no test on this path, so no
reference output pins either restatement.  This twin exists to catch logic
errors in the C oracle (ordering, Schur blocks, LM bookkeeping, Huber gate,
rollback semantics); it shares no code with it.  It is vectorised over edges
and uses numpy's summation order, so it agrees with the C oracle to rounding
(not bitwise).  Only tests/ and tests/golden/make_golden.py import it.

Follows (reference paths under src/ and include/):
  solve loop                 src/lego/base/problem.cpp:156-230
  ordering (SLAM)            src/lego/base/problem.cpp:234-255, :48-58
  buildHessian               src/lego/base/problem.cpp:273-358
  solveLinearEquation, SLAM  src/lego/base/problem.cpp:380-430  (dense, as written)
  updateStates / rollback    src/lego/base/problem.cpp:433-467
  computeLambdaInitLM        src/lego/base/problem.cpp:470-504
  isGoodStepInLM             src/lego/base/problem.cpp:520-581
  getChi2 / getRobustChi2 / computeRobustInformation
                             src/lego/base/base_edge.cpp:31-64
  HuberCost::compute         src/lego/base/cost_function.cpp:5-17
  EdgeProjection residual / Jacobians
                             include/legoslam/lego_types.h:200-254
  VertexPose::add / VertexXYZ::add
                             include/legoslam/lego_types.h:61-91, :105-112
  Eigen LDLT (diagonal pivoting, pseudo-inverse solve), PartialPivLU inverse,
  Sophus SE3::exp / SE3(Matrix4) / SE3 * SE3   (third-party, versions unpinned)

Window layout (lego_ba.generate_window): pose_Tcw (P,12) row-major [R|t],
lm_xyz (L,3), obs_pose/obs_lm (O,) uint32, obs_cam (O,) uint8, obs_uv (O,2),
K = (fx, fy, cx, cy), cam_ext (ncam,12), optional pose_fixed (P,) uint8.
Poses are in ascending keyframe id and landmarks in ascending landmark id, which
is the reference's ordering (problem.cpp:234-255).
"""
import numpy as np

SOPHUS_EPS = 1e-10                       # Sophus Constants<double>::epsilon()
DBL_MIN = np.finfo(np.float64).tiny      # numeric_limits<double>::min() (LDLT solve cutoff)


# --------------------------------------------------------------------------
# Sophus / Eigen pieces (vectorised over a leading axis where useful)
# --------------------------------------------------------------------------

def quat_from_rot(R):
    """Eigen Quaternion(Matrix3) (Shepperd's method, trace branch first).  q = (w, x, y, z)."""
    t = R[0, 0] + R[1, 1] + R[2, 2]
    if t > 0.0:
        s = np.sqrt(t + 1.0)
        w = 0.5 * s
        s = 0.5 / s
        return np.array([w, (R[2, 1] - R[1, 2]) * s, (R[0, 2] - R[2, 0]) * s, (R[1, 0] - R[0, 1]) * s])
    i = 0
    if R[1, 1] > R[0, 0]:
        i = 1
    if R[2, 2] > R[i, i]:
        i = 2
    j, k = (i + 1) % 3, (i + 2) % 3
    s = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
    v = np.zeros(3)
    v[i] = 0.5 * s
    s = 0.5 / s
    v[j] = (R[j, i] + R[i, j]) * s
    v[k] = (R[k, i] + R[i, k]) * s
    return np.array([(R[k, j] - R[j, k]) * s, v[0], v[1], v[2]])


def rot_from_quat(q):
    """Eigen QuaternionBase::toRotationMatrix."""
    w, x, y, z = q
    return np.array([
        [1.0 - 2.0 * (y * y + z * z), 2.0 * (x * y - w * z), 2.0 * (x * z + w * y)],
        [2.0 * (x * y + w * z), 1.0 - 2.0 * (x * x + z * z), 2.0 * (y * z - w * x)],
        [2.0 * (x * z - w * y), 2.0 * (y * z + w * x), 1.0 - 2.0 * (x * x + y * y)],
    ])


def quat_mul(a, b):
    """Quaternion product, then Sophus SO3 renormalisation (squared norm around 1)."""
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    q = np.array([aw * bw - ax * bx - ay * by - az * bz,
                  aw * bx + ax * bw + ay * bz - az * by,
                  aw * by + ay * bw + az * bx - ax * bz,
                  aw * bz + az * bw + ax * by - ay * bx])
    sq = float(q @ q)
    if sq != 1.0:
        q = q * (2.0 / (1.0 + sq))
    return q


def se3_exp(a):
    """Sophus SE3::exp of the twist a = (upsilon, omega): translation first."""
    ups, om = np.asarray(a[:3], float), np.asarray(a[3:], float)
    th2 = float(om @ om)
    th = np.sqrt(th2)
    if th < SOPHUS_EPS:
        imag = 0.5 - th2 / 48.0 + th2 * th2 / 3840.0
        real = 1.0 - th2 / 8.0 + th2 * th2 / 384.0
    else:
        imag = np.sin(0.5 * th) / th
        real = np.cos(0.5 * th)
    q = np.array([real, imag * om[0], imag * om[1], imag * om[2]])
    if th < SOPHUS_EPS:
        V = rot_from_quat(q)
    else:
        Om = np.array([[0.0, -om[2], om[1]], [om[2], 0.0, -om[0]], [-om[1], om[0], 0.0]])
        V = np.eye(3) + (1.0 - np.cos(th)) / th2 * Om + (th - np.sin(th)) / (th2 * th) * (Om @ Om)
    return q, V @ ups


def pose_left_update(T12, d):
    """VertexPose::add: estimate_ <- (SE3::exp(d) * SE3(estimate_)).matrix(); a NaN/Inf
    component zeroes the whole update (lego_types.h:63-69)."""
    d = np.asarray(d, float)
    if not np.all(np.isfinite(d)):
        d = np.zeros(6)
    qe, te = se3_exp(d)
    T = np.asarray(T12, float).reshape(3, 4)
    qt = quat_from_rot(T[:, :3])
    q = quat_mul(qe, qt)
    t = te + rot_from_quat(qe) @ T[:, 3]
    out = np.empty((3, 4))
    out[:, :3] = rot_from_quat(q)
    out[:, 3] = t
    return out.reshape(12)


def sophus_pose(T12):
    """SE3(estimate_): the 4x4 goes through a quaternion (lego_types.h:211, :229)."""
    T = np.asarray(T12, float).reshape(3, 4)
    return rot_from_quat(quat_from_rot(T[:, :3])), T[:, 3].copy()


def eigen_ldlt_solve(A, b):
    """Eigen LDLT<MatrixXd, Lower>::compute + solve: left-looking, pivoting on the largest
    remaining diagonal entry (the not-yet-updated one), zero pivots skipped, solve with the
    pseudo-inverse of D (|d| <= DBL_MIN -> 0).  Reads the lower triangle only."""
    n = A.shape[0]
    M = np.tril(np.array(A, dtype=float))
    M = M + np.tril(M, -1).T          # symmetric from the lower triangle (what Eigen reads)
    perm = np.arange(n)
    trans = np.arange(n)
    L = np.zeros((n, n))
    d = np.zeros(n)
    for k in range(n):
        j = k + int(np.argmax(np.abs(np.diag(M)[k:])))
        trans[k] = j
        if j != k:
            M[[k, j], :] = M[[j, k], :]
            M[:, [k, j]] = M[:, [j, k]]
            L[[k, j], :k] = L[[j, k], :k]
            perm[[k, j]] = perm[[j, k]]
        # left-looking update of column k
        akk = M[k, k] - (L[k, :k] * d[:k]) @ L[k, :k]
        col = M[k + 1:, k] - L[k + 1:, :k] @ (d[:k] * L[k, :k])
        if k == 0 and akk == 0.0:
            # all-zero diagonal: Eigen stops, L = I, D = diag(M)
            d = np.diag(M).copy()
            L = np.eye(n)
            trans = np.arange(n)
            break
        d[k] = akk
        L[k, k] = 1.0
        L[k + 1:, k] = col / akk if akk != 0.0 else col
        # the remaining diagonal keeps its ORIGINAL (unupdated) values for pivot selection,
        # exactly as the in-place matrix does in Eigen's left-looking loop
    x = np.array(b, dtype=float)
    for k in range(n):
        j = trans[k]
        if j != k:
            x[[k, j]] = x[[j, k]]
    for k in range(n):                        # L y = P b
        x[k + 1:] -= L[k + 1:, k] * x[k]
    x = np.where(np.abs(d) > DBL_MIN, x / np.where(d == 0.0, 1.0, d), 0.0)
    for k in range(n - 1, -1, -1):            # L^T z = y
        x[:k] -= L[k, :k] * x[k]
    for k in range(n - 1, -1, -1):
        j = trans[k]
        if j != k:
            x[[k, j]] = x[[j, k]]
    return x


def huber(e2, delta):
    """HuberCost::compute, vectorised: (rho0, rho1, rho2)."""
    e2 = np.asarray(e2, float)
    if delta is None or delta <= 0.0:
        return e2.copy(), np.ones_like(e2), np.zeros_like(e2)
    d2 = delta * delta
    inl = e2 <= d2
    s = np.sqrt(np.where(inl, 1.0, e2))
    r0 = np.where(inl, e2, 2.0 * s * delta - d2)
    r1 = np.where(inl, 1.0, delta / s)
    r2 = np.where(inl, 0.0, -0.5 * r1 / np.where(inl, 1.0, e2))
    return r0, r1, r2


# --------------------------------------------------------------------------
# the problem
# --------------------------------------------------------------------------

class Problem:
    """lego::Problem(SLAM) with EdgeProjection edges and a Huber cost (backend_lego.cpp:56-161)."""

    def __init__(self, w, huber_delta=5.991, strategy=0, tau=1e-5, lambda_cap=5e10, lambda_init=None,
                 stop_dchi2=1e-5, max_trials=10, gate_mode=0):
        self.P = int(np.asarray(w["pose_Tcw"]).shape[0])
        self.L = int(np.asarray(w["lm_xyz"]).shape[0])
        self.pose = np.array(w["pose_Tcw"], float).reshape(self.P, 12)
        self.lm = np.array(w["lm_xyz"], float).reshape(self.L, 3)
        self.op = np.asarray(w["obs_pose"]).astype(np.int64)
        self.ol = np.asarray(w["obs_lm"]).astype(np.int64)
        self.O = self.op.shape[0]
        oc = w.get("obs_cam")
        self.oc = np.zeros(self.O, np.int64) if oc is None else np.asarray(oc).astype(np.int64)
        self.uv = np.array(w["obs_uv"], float).reshape(self.O, 2)
        self.K = np.asarray(w["K"], float)
        ext = w.get("cam_ext")
        if ext is None:
            ext = np.array([[1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0]], float)
        self.ext = [sophus_pose(e) for e in np.asarray(ext, float).reshape(-1, 12)]
        fx = w.get("pose_fixed")
        self.fixed = np.zeros(self.P, bool) if fx is None else np.asarray(fx).astype(bool)
        self.delta = huber_delta
        self.strategy = strategy
        self.tau, self.lambda_cap, self.lambda_init = tau, lambda_cap, lambda_init
        self.stop_dchi2, self.max_trials = stop_dchi2, max_trials
        # 0: the reference Huber gate (base_edge.cpp:55), whose sign for an outlier edge is a
        # rounding residue; 1: that residue taken as 0 (the C oracle's gate_mode 1).  The twin is
        # not bitwise, so on windows with outliers it is compared with the C oracle in mode 1.
        self.gate_mode = gate_mode
        self.np_ = 6 * self.P
        self.n = self.np_ + 3 * self.L
        self.res = np.zeros((self.O, 2))

    # ---- EdgeProjection -------------------------------------------------
    def _poses(self):
        return [sophus_pose(self.pose[p]) for p in range(self.P)]

    def residuals(self):
        """computeResidual for every edge: r = z - pi(K (ext (T X)))  (lego_types.h:211-215)."""
        Ts = self._poses()
        R = np.stack([t[0] for t in Ts])[self.op]
        t = np.stack([t[1] for t in Ts])[self.op]
        Re = np.stack([e[0] for e in self.ext])[self.oc]
        te = np.stack([e[1] for e in self.ext])[self.oc]
        X = self.lm[self.ol]
        Pb = np.einsum("eij,ej->ei", R, X) + t
        Pc = np.einsum("eij,ej->ei", Re, Pb) + te
        fx, fy, cx, cy = self.K
        u = (fx * Pc[:, 0] + cx * Pc[:, 2]) / (Pc[:, 2] + 1e-18)
        v = (fy * Pc[:, 1] + cy * Pc[:, 2]) / (Pc[:, 2] + 1e-18)
        return self.uv - np.stack([u, v], axis=1)

    def jacobians(self):
        """computeJacobians (lego_types.h:218-254): J_p (2x6, [rho; phi]) at (ext T) X and
        J_l = J_p[:, :3] R_ext R_T."""
        Ts = self._poses()
        R = np.stack([t[0] for t in Ts])
        t = np.stack([t[1] for t in Ts])
        Re = np.stack([e[0] for e in self.ext])
        te = np.stack([e[1] for e in self.ext])
        # composed transform ext * T, per (camera, pose), then applied to X
        Rc = np.einsum("cij,pjk->cpik", Re, R)
        tc = np.einsum("cij,pj->cpi", Re, t) + te[:, None, :]
        X = self.lm[self.ol]
        Pc = np.einsum("eij,ej->ei", Rc[self.oc, self.op], X) + tc[self.oc, self.op]
        fx, fy = self.K[0], self.K[1]
        x, y, z = Pc[:, 0], Pc[:, 1], Pc[:, 2]
        zi = 1.0 / (z + 1e-18)
        zi2 = zi * zi
        Jp = np.zeros((self.O, 2, 6))
        Jp[:, 0, 0] = -fx * zi
        Jp[:, 0, 2] = fx * x * zi2
        Jp[:, 0, 3] = fx * x * y * zi2
        Jp[:, 0, 4] = -fx - fx * x * x * zi2
        Jp[:, 0, 5] = fx * y * zi
        Jp[:, 1, 1] = -fy * zi
        Jp[:, 1, 2] = fy * y * zi2
        Jp[:, 1, 3] = fy + fy * y * y * zi2
        Jp[:, 1, 4] = -fy * x * y * zi2
        Jp[:, 1, 5] = -fy * x * zi
        Jl = np.einsum("eij,ejk->eik", Jp[:, :, :3], Rc[self.oc, self.op])
        return Jp, Jl

    def robust_chi2(self, res):
        e2 = np.einsum("ei,ei->e", res, res)
        return huber(e2, self.delta)[0]

    # ---- Problem --------------------------------------------------------
    def build_hessian(self):
        """buildHessian: dense H (n x n) and b, fixed vertices contribute nothing."""
        self.res = self.residuals()
        Jp, Jl = self.jacobians()
        e2 = np.einsum("ei,ei->e", self.res, self.res)
        _, r1, r2 = huber(e2, self.delta)
        W = r1[:, None, None] * np.eye(2)[None]
        gate = (r1 + 2.0 * r2 * e2) > 0.0
        if self.gate_mode == 1 and self.delta is not None and self.delta > 0.0:
            gate &= ~(e2 > self.delta * self.delta)    # diagnostic: the analytically-zero residue is 0
        W = W + np.where(gate, 2.0 * r2, 0.0)[:, None, None] * np.einsum("ei,ej->eij", self.res, self.res)
        live = ~self.fixed[self.op]
        Hpp = np.einsum("eai,eab,ebj->eij", Jp, W, Jp)
        Hpl = np.einsum("eai,eab,ebj->eij", Jp, W, Jl)
        Hll = np.einsum("eai,eab,ebj->eij", Jl, W, Jl)
        bp = -r1[:, None] * np.einsum("eai,ea->ei", Jp, self.res)
        bl = -r1[:, None] * np.einsum("eai,ea->ei", Jl, self.res)
        H = np.zeros((self.n, self.n))
        b = np.zeros(self.n)
        pi = 6 * self.op
        li = self.np_ + 3 * self.ol
        for e in range(self.O):
            p, l = pi[e], li[e]
            if live[e]:
                H[p:p + 6, p:p + 6] += Hpp[e]
                H[p:p + 6, l:l + 3] += Hpl[e]
                H[l:l + 3, p:p + 6] += Hpl[e].T
                b[p:p + 6] += bp[e]
            H[l:l + 3, l:l + 3] += Hll[e]
            b[l:l + 3] += bl[e]
        self.H, self.b = H, b
        self.dx = np.zeros(self.n)

    def solve_linear(self):
        """solveLinearEquation, SLAM branch, dense as written (problem.cpp:380-430)."""
        m = self.np_
        H, b = self.H, self.b
        Hmm = H[m:, m:]
        Hmm_inv = np.zeros_like(Hmm)
        for l in range(self.L):
            s = slice(3 * l, 3 * l + 3)
            with np.errstate(all="ignore"):
                try:
                    Hmm_inv[s, s] = np.linalg.inv(Hmm[s, s])
                except np.linalg.LinAlgError:
                    Hmm_inv[s, s] = np.inf
        tempH = H[:m, m:] @ Hmm_inv
        S = H[:m, :m] - tempH @ H[m:, :m]
        bs = b[:m] - tempH @ b[m:]
        idx = np.arange(m)
        if self.strategy == 0:
            S[idx, idx] += self.lam
        else:
            S[idx, idx] += self.lam * S[idx, idx]
        dxp = eigen_ldlt_solve(S, bs)
        dxl = Hmm_inv @ (b[m:] - H[m:, :m] @ dxp)
        self.dx = np.concatenate([dxp, dxl])

    def update_states(self):
        self.pose_bak, self.lm_bak = self.pose.copy(), self.lm.copy()
        for p in range(self.P):
            self.pose[p] = pose_left_update(self.pose[p], self.dx[6 * p:6 * p + 6])
        d = self.dx[self.np_:].reshape(self.L, 3)
        ok = np.all(np.isfinite(d), axis=1)
        self.lm[ok] += d[ok]

    def rollback_states(self):
        self.pose, self.lm = self.pose_bak.copy(), self.lm_bak.copy()

    def lambda_init_lm(self):
        self.ni = 2.0
        self.chi = 0.5 * float(np.sum(self.robust_chi2(self.res)))
        if self.strategy == 0:
            if self.lambda_init is None:
                m = min(self.lambda_cap, float(np.max(np.abs(np.diag(self.H)), initial=0.0)))
                self.lam = self.tau * m
            else:
                self.lam = self.lambda_init
        else:
            self.lam = 1e-5

    def good_step(self):
        self.res = self.residuals()
        temp = 0.5 * float(np.sum(self.robust_chi2(self.res)))
        if self.strategy == 0:
            scale = 0.5 * float(self.dx @ (self.lam * self.dx + self.b)) + 1e-10
            rho = (self.chi - temp) / scale
            if rho > 0 and np.isfinite(temp):
                alpha = min(1.0 - (2 * rho - 1) ** 3, 2.0 / 3.0)
                self.lam *= max(1.0 / 3.0, alpha)
                self.ni = 2.0
                self.chi = temp
                return True
            self.lam *= self.ni
            self.ni *= 2
            return False
        scale = 0.5 * float(self.dx @ (self.lam * np.diag(self.H) * self.dx + self.b)) + 1e-10
        rho = (self.chi - temp) / scale
        if rho > 0 and np.isfinite(temp):
            self.lam = max(self.lam / 9.0, 1e-7)
            self.chi = temp
            return True
        self.lam = min(self.lam * 11.0, 1e7)
        return False

    def solve(self, iterations=10):
        """Problem::solve(iterations).  Returns None for an empty problem (problem.cpp:157-161)."""
        if self.O == 0 or self.P + self.L == 0:
            return None
        self.build_hessian()
        self.lambda_init_lm()
        chi0 = self.chi
        trace = []      # (chi, lambda) at the top of each iteration (the verbose line, problem.cpp:180-184)
        it, trials, last = 0, 0, 1e20
        stop = False
        while not stop and it < iterations:
            trace.append((self.chi, self.lam))
            ok, false_cnt = False, 0
            while not ok and false_cnt < self.max_trials:
                self.solve_linear()
                self.update_states()
                ok = self.good_step()
                trials += 1
                if ok:
                    self.build_hessian()
                else:
                    false_cnt += 1
                    self.rollback_states()
            it += 1
            if last - self.chi < self.stop_dchi2:
                stop = True
            last = self.chi
        # edge robust chi2 "as last evaluated" 
        return dict(pose_Tcw=self.pose.copy(), lm_xyz=self.lm.copy(), chi2_initial=chi0, chi2_final=self.chi,
                    lambda_final=self.lam, iterations=it, trials=trials,
                    edge_robust_chi2=self.robust_chi2(self.res),
                    trace_chi2=np.array([c for c, _ in trace]), trace_lambda=np.array([l for _, l in trace]))


def solve(w, max_iters=10, **kw):
    """Backend::Optimize's problem.solve(max_iters) on window `w`."""
    return Problem(w, **kw).solve(max_iters)

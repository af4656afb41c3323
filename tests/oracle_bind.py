"""
oracle_bind — ctypes binding to oracle/liblego_oracle.so (TEST INFRASTRUCTURE).

The oracle is the checker: a CPU restatement of the reference solve
(oracle/lego_oracle.c).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use it.  Parity is unpinned (see oracle/lego_oracle.c header).
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_LIB = os.environ.get("LH_ORACLE_LIB") or os.path.join(ROOT, "oracle", "liblego_oracle.so")   # (env: sanitizer builds)


class OrcOptions(C.Structure):
    _fields_ = [
        ("max_iters", C.c_int32), ("max_trials", C.c_int32), ("strategy", C.c_int32),
        ("verbose", C.c_int32), ("n_threads", C.c_int32), ("gate_mode", C.c_int32),
        ("huber_delta", C.c_double), ("stop_dchi2", C.c_double), ("tau", C.c_double),
        ("lambda_cap", C.c_double), ("lambda_init", C.c_double),
        ("linear_solver", C.c_int32), ("pcg_max_iters", C.c_int32), ("pcg_tol", C.c_double),
        ("degenerate_guard", C.c_int32), ("pad_", C.c_int32),
    ]


class OrcStats(C.Structure):
    _fields_ = [
        ("chi2_initial", C.c_double), ("chi2_final", C.c_double), ("lambda_final", C.c_double),
        ("time_ms", C.c_double), ("iterations", C.c_int32), ("trials", C.c_int32),
        ("accepted", C.c_int32), ("trace_len", C.c_int32),
        ("pcg_iterations", C.c_int32), ("pad_", C.c_int32),
    ]


_libs = {}


def lib(path=None):
    """The oracle library (default: oracle/liblego_oracle.so, the parity build); `path` loads another
    build of the same source (bench.py's -O3 -march=native cpu_baseline build)."""
    path = path or ORACLE_LIB
    if path not in _libs:
        if path == ORACLE_LIB and not os.path.exists(ORACLE_LIB):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(path)
        vp = C.c_void_p
        L.orc_solve.argtypes = [C.c_int, C.c_int32, vp, vp, C.c_int32, vp, C.c_int64, vp, vp, vp, vp, vp,
                                C.c_int32, vp, C.POINTER(OrcOptions), vp, vp, vp, vp, vp, C.c_int32,
                                C.POINTER(OrcStats)]
        L.orc_solve.restype = C.c_int
        L.orc_reduced_system.argtypes = [C.c_int32, vp, vp, C.c_int32, vp, C.c_int64, vp, vp, vp, vp, vp,
                                         C.c_int32, vp, C.POINTER(OrcOptions), vp, vp, vp]
        L.orc_reduced_system.restype = C.c_int
        L.orc_se3_exp.argtypes = [vp, vp]
        L.orc_se3_left_update.argtypes = [vp, vp, vp]
        L.orc_huber.argtypes = [C.c_double, C.c_double, vp]
        L.orc_lu_inverse3.argtypes = [vp, vp]
        L.orc_ldlt_solve.argtypes = [vp, C.c_int, vp, vp]
        L.orc_pcg_solve.argtypes = [vp, C.c_int, vp, vp, C.c_double, C.c_int]
        L.orc_pcg_solve.restype = C.c_int
        L.orc_edge_eval.argtypes = [vp] * 5 + [C.c_double] + [vp] * 6
        _libs[path] = L
    return _libs[path]


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def options(max_iters=10, max_trials=10, strategy=0, huber_delta=5.991, stop_dchi2=1e-5, tau=1e-5,
            lambda_cap=5e10, lambda_init=-1.0, verbose=0, n_threads=0, gate_mode=0, linear_solver=0,
            pcg_max_iters=0, pcg_tol=1e-6, degenerate_guard=0):
    return OrcOptions(max_iters, max_trials, strategy, verbose, n_threads, gate_mode, huber_delta, stop_dchi2,
                      tau, lambda_cap, lambda_init, linear_solver, pcg_max_iters, pcg_tol, degenerate_guard, 0)


def solve(w, variant=1, trace_cap=64, lib_path=None, **opt):
    """Run the oracle on window dict `w` (lego_ba.generate_window layout)."""
    a = lambda k, dt: None if w.get(k) is None else np.ascontiguousarray(w[k], dtype=dt)
    pose, lm = a("pose_Tcw", np.float64), a("lm_xyz", np.float64)
    op, ol, oc, uv = a("obs_pose", np.uint32), a("obs_lm", np.uint32), a("obs_cam", np.uint8), a("obs_uv", np.float64)
    fixed, ext = a("pose_fixed", np.uint8), a("cam_ext", np.float64)
    K = np.ascontiguousarray(w["K"], np.float64)
    P, L, O = pose.shape[0], lm.shape[0], op.shape[0]
    out = dict(pose_Tcw=np.zeros((P, 12)), lm_xyz=np.zeros((L, 3)), edge_robust_chi2=np.zeros(O),
               trace_chi2=np.zeros(trace_cap), trace_lambda=np.zeros(trace_cap))
    st = OrcStats()
    o = options(**opt)
    rc = lib(lib_path).orc_solve(variant, P, _p(pose), _p(fixed), L, _p(lm), O, _p(op), _p(ol), _p(oc), _p(uv), _p(K),
                         0 if ext is None else ext.shape[0], _p(ext), C.byref(o), _p(out["pose_Tcw"]),
                         _p(out["lm_xyz"]), _p(out["edge_robust_chi2"]), _p(out["trace_chi2"]),
                         _p(out["trace_lambda"]), trace_cap, C.byref(st))
    out["status"] = rc
    out["trace_chi2"] = out["trace_chi2"][:st.trace_len]
    out["trace_lambda"] = out["trace_lambda"][:st.trace_len]
    for f in ("chi2_initial", "chi2_final", "lambda_final", "time_ms", "iterations", "trials", "accepted",
              "pcg_iterations"):
        out[f] = getattr(st, f)
    return out


def reduced_system(w, **opt):
    """Undamped reduced pose system (S, bs) and sum rho0 of window `w` at its input state
    (oracle/lego_oracle.c orc_reduced_system)."""
    a = lambda k, dt: None if w.get(k) is None else np.ascontiguousarray(w[k], dtype=dt)
    pose, lm = a("pose_Tcw", np.float64), a("lm_xyz", np.float64)
    op, ol, oc, uv = a("obs_pose", np.uint32), a("obs_lm", np.uint32), a("obs_cam", np.uint8), a("obs_uv", np.float64)
    fixed, ext = a("pose_fixed", np.uint8), a("cam_ext", np.float64)
    K = np.ascontiguousarray(w["K"], np.float64)
    P, L, O = pose.shape[0], lm.shape[0], op.shape[0]
    S = np.zeros((6 * P, 6 * P))
    bs = np.zeros(6 * P)
    chi2 = C.c_double(0.0)
    o = options(**opt)
    rc = lib().orc_reduced_system(P, _p(pose), _p(fixed), L, _p(lm), O, _p(op), _p(ol), _p(oc), _p(uv), _p(K),
                                  0 if ext is None else ext.shape[0], _p(ext), C.byref(o), _p(S), _p(bs),
                                  C.byref(chi2))
    assert rc == 0, rc
    return S, bs, chi2.value


def landmark_shard(w, l0, l1):
    """The sub-window of landmarks [l0, l1) and their observations (poses replicated), the
    unit one GPU owns in the landmark-sharded multi-GPU path."""
    keep = (w["obs_lm"] >= l0) & (w["obs_lm"] < l1)
    s = dict(w)
    s["lm_xyz"] = w["lm_xyz"][l0:l1]
    s["obs_lm"] = (w["obs_lm"][keep] - l0).astype(np.uint32)
    for k in ("obs_pose", "obs_cam", "obs_uv"):
        if w.get(k) is not None:
            s[k] = w[k][keep]
    return s


def se3_exp(a):
    T = np.zeros(12)
    lib().orc_se3_exp(_p(np.ascontiguousarray(a, np.float64)), _p(T))
    return T


def se3_left_update(a, T12):
    out = np.zeros(12)
    lib().orc_se3_left_update(_p(np.ascontiguousarray(a, np.float64)), _p(np.ascontiguousarray(T12, np.float64)), _p(out))
    return out


def huber(delta, e2):
    rho = np.zeros(3)
    lib().orc_huber(delta, e2, _p(rho))
    return rho


def lu_inverse3(A):
    out = np.zeros(9)
    lib().orc_lu_inverse3(_p(np.ascontiguousarray(A, np.float64).reshape(9)), _p(out))
    return out.reshape(3, 3)


def ldlt_solve(A, b):
    A = np.ascontiguousarray(A, np.float64)
    x = np.zeros(A.shape[0])
    lib().orc_ldlt_solve(_p(A), A.shape[0], _p(np.ascontiguousarray(b, np.float64)), _p(x))
    return x


def estimate_pose(fb, is_outlier_in=None, **opt):
    """Frontend::EstimateCurrentPose on every frame of batch `fb` (tests/frames.py layout)."""
    L = lib()
    vp = C.c_void_p
    L.orc_estimate_pose.argtypes = [C.c_int32, vp, vp, vp, vp, vp, C.POINTER(OrcOptions), vp, vp, vp, vp, vp, vp]
    L.orc_estimate_pose.restype = C.c_int
    F = int(fb["n_frames"])
    O = int(fb["obs_ptr"][-1])
    ptr = np.ascontiguousarray(fb["obs_ptr"], np.int64)
    pose = np.ascontiguousarray(fb["pose_Tcw"], np.float64).reshape(F, 12)
    pts = np.ascontiguousarray(fb["pts"], np.float64)
    uv = np.ascontiguousarray(fb["obs_uv"], np.float64)
    K = np.ascontiguousarray(fb["K"], np.float64)
    fin = None if is_outlier_in is None else np.ascontiguousarray(is_outlier_in, np.uint8)
    out = dict(pose_Tcw=np.zeros((F, 12)), is_outlier=np.zeros(O, np.uint8), rchi2=np.zeros(O),
               iterations=np.zeros(F, np.int32), trials=np.zeros(F, np.int32))
    o = options(**opt)
    rc = L.orc_estimate_pose(F, _p(ptr), _p(pose), _p(pts), _p(uv), _p(K), C.byref(o), _p(fin), _p(out["pose_Tcw"]),
                             _p(out["is_outlier"]), _p(out["rchi2"]), _p(out["iterations"]), _p(out["trials"]))
    assert rc == 0, rc
    out["is_outlier"] = out["is_outlier"].astype(bool)
    return out


def pcg_solve(A, b, tol=1e-6, max_iters=0):
    """The fixed reference PCG (oracle pcg_solve): (x, steps)."""
    A = np.ascontiguousarray(A, np.float64)
    x = np.zeros(A.shape[0])
    it = lib().orc_pcg_solve(_p(A), A.shape[0], _p(np.ascontiguousarray(b, np.float64)), _p(x), tol, max_iters)
    return x, it


def edge_eval(T12, X, uv, K, ext12=None, huber_delta=5.991):
    if ext12 is None:
        ext12 = np.array([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0], np.float64)
    r, Jp, Jl, W = np.zeros(2), np.zeros(12), np.zeros(6), np.zeros(4)
    drho, rc = C.c_double(), C.c_double()
    f = lambda v: _p(np.ascontiguousarray(v, np.float64))
    lib().orc_edge_eval(f(T12), f(X), f(uv), f(K), f(ext12), huber_delta, _p(r), _p(Jp), _p(Jl), _p(W),
                        C.byref(drho), C.byref(rc))
    return dict(r=r, Jp=Jp.reshape(2, 6), Jl=Jl.reshape(2, 3), W=W.reshape(2, 2), drho=drho.value, rchi2=rc.value)


def lk_track(img1, img2, kp1, kp2_init=None, inverse=False, levels=4, lib_path=None):
    """orc_lk_track: the restated LKOpticalFlow4Layer / 1Layer (oracle/lk_oracle.c)."""
    L = lib(lib_path)
    L.orc_lk_track.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int64, C.c_int32, C.c_void_p,
                               C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32]
    L.orc_lk_track.restype = C.c_int
    i1 = np.ascontiguousarray(img1, dtype=np.uint8)
    i2 = np.ascontiguousarray(img2, dtype=np.uint8)
    k1 = np.ascontiguousarray(kp1, dtype=np.float32).reshape(-1, 2)
    n = k1.shape[0]
    k2 = (np.zeros((n, 2), np.float32) if kp2_init is None
          else np.array(kp2_init, dtype=np.float32, copy=True).reshape(-1, 2))
    ok = np.zeros(n, np.uint8)
    rows, cols = i1.shape
    rc = L.orc_lk_track(i1.ctypes.data, i2.ctypes.data, cols, rows, i1.strides[0], n, k1.ctypes.data, k2.ctypes.data,
                        ok.ctypes.data, int(bool(inverse)), int(kp2_init is not None), int(levels))
    if rc != 0:
        raise ValueError(f"orc_lk_track: {rc}")
    return dict(kp2=k2, success=ok.astype(bool))


def lk_pyr_down(src, dw, dh):
    L = lib()
    L.orc_lk_pyr_down.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int64, C.c_void_p, C.c_int32, C.c_int32]
    s = np.ascontiguousarray(src, dtype=np.uint8)
    d = np.zeros((dh, dw), np.uint8)
    L.orc_lk_pyr_down(s.ctypes.data, s.shape[1], s.shape[0], s.strides[0], d.ctypes.data, dw, dh)
    return d

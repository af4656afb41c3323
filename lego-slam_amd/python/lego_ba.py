"""
lego_ba — ctypes bindings for the MI355X BA solver C ABI (include/lego_ba.h)
and for the synthetic window generator (lego-slam_amd/tools/lh_window.h).

This is plumbing for tests/bench: the product is liblego_ba.so (HIP kernels +
C ABI); this module only marshals numpy arrays across that boundary.  It never
falls back to a CPU path: if liblego_ba.so is missing, Solver() raises.
"""
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # lego-slam_amd/
LIB_DIR = os.path.join(PKG_DIR, "lib")
BA_LIB = os.environ.get("LH_LIB") or os.path.join(LIB_DIR, "liblego_ba.so")
WIN_LIB = os.environ.get("LH_WIN_LIB") or os.path.join(LIB_DIR, "liblego_window.so")   # (env: sanitizer builds)

# --------------------------------------------------------------------------
# window generator
# --------------------------------------------------------------------------


class LhwParams(C.Structure):
    _fields_ = [
        ("n_poses", C.c_int32), ("n_landmarks", C.c_int32),
        ("k_min", C.c_int32), ("k_max", C.c_int32),
        ("pose_mode", C.c_int32), ("seed", C.c_uint64),
        ("noise_px", C.c_double), ("outlier_frac", C.c_double),
        ("right_frac", C.c_double), ("baseline", C.c_double),
        ("step_m", C.c_double), ("yaw_sigma", C.c_double),
        ("depth_min", C.c_double), ("depth_max", C.c_double),
        ("pose_rot_sigma", C.c_double), ("pose_trans_sigma", C.c_double),
        ("lm_sigma", C.c_double), ("K", C.c_double * 4),
        ("width", C.c_double), ("height", C.c_double),
    ]


_winlib = None


def _wl():
    global _winlib
    if _winlib is None:
        if not os.path.exists(WIN_LIB):
            raise RuntimeError(f"{WIN_LIB} not built (run __graft_entry__.build())")
        lib = C.CDLL(WIN_LIB)
        lib.lhw_default_params.argtypes = [C.POINTER(LhwParams)]
        lib.lhw_count_obs.argtypes = [C.POINTER(LhwParams), C.c_int32, C.c_int32]
        lib.lhw_count_obs.restype = C.c_int64
        lib.lhw_poses.argtypes = [C.POINTER(LhwParams), C.c_void_p, C.c_void_p]
        lib.lhw_cameras.argtypes = [C.POINTER(LhwParams), C.c_void_p]
        lib.lhw_landmarks.argtypes = [C.POINTER(LhwParams), C.c_int32, C.c_int32] + [C.c_void_p] * 6
        lib.lhw_landmarks.restype = C.c_int64
        _winlib = lib
    return _winlib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


# Named configurations (BASELINE.json "configs").
CONFIGS = {
    "C1": dict(P=5, L=200, k=5),        # CPU plumbing window
    "mini": dict(P=10, L=500, k=8),
    "C2": dict(P=10, L=5000, k=8),
    "C3": dict(P=20, L=50000, k=8),     # bench workload (metric window)
    "C4": dict(P=20, L=500000, k=8),    # 8-GPU window
    "W32": dict(P=32, L=3000, k=8),     # past 21 keyframes: the reduced system in global memory (k_ctrl_g)
    "W24s": dict(P=24, L=500, k=8),     # a small window past 21 keyframes (golden fixture)
}


def window_params(P=20, L=50000, k=8, k_max=None, seed=0, **kw):
    p = LhwParams()
    _wl().lhw_default_params(C.byref(p))
    p.n_poses, p.n_landmarks, p.k_min = P, L, k
    p.k_max = k if k_max is None else k_max
    p.seed = seed
    for name, v in kw.items():
        if name == "K":
            for i in range(4):
                p.K[i] = v[i]
        else:
            setattr(p, name, v)
    return p


def generate_window(P=20, L=50000, k=8, seed=0, lm_begin=0, lm_end=None, **kw):
    """Generate landmarks [lm_begin, lm_end) of a synthetic window (all poses)."""
    p = window_params(P=P, L=L, k=k, seed=seed, **kw)
    lib = _wl()
    lm_end = L if lm_end is None else lm_end
    n_lm = lm_end - lm_begin
    n_obs = lib.lhw_count_obs(C.byref(p), lm_begin, lm_end)
    w = dict(
        n_poses=P,
        pose_true=np.zeros((P, 12)), pose_Tcw=np.zeros((P, 12)),
        lm_true=np.zeros((n_lm, 3)), lm_xyz=np.zeros((n_lm, 3)),
        obs_pose=np.zeros(n_obs, np.uint32), obs_lm=np.zeros(n_obs, np.uint32),
        obs_cam=np.zeros(n_obs, np.uint8), obs_uv=np.zeros((n_obs, 2)),
        cam_ext=np.zeros((2, 12)), K=np.array(list(p.K)),
    )
    lib.lhw_poses(C.byref(p), _ptr(w["pose_true"]), _ptr(w["pose_Tcw"]))
    lib.lhw_cameras(C.byref(p), _ptr(w["cam_ext"]))
    got = lib.lhw_landmarks(C.byref(p), lm_begin, lm_end, _ptr(w["lm_true"]), _ptr(w["lm_xyz"]),
                            _ptr(w["obs_pose"]), _ptr(w["obs_lm"]), _ptr(w["obs_cam"]), _ptr(w["obs_uv"]))
    assert got == n_obs, (got, n_obs)
    return w


def config_window(name, seed=0, **kw):
    c = dict(CONFIGS[name])
    c.update(kw)
    return generate_window(seed=seed, **c)


# --------------------------------------------------------------------------
# solver C ABI (include/lego_ba.h)
# --------------------------------------------------------------------------

LH_OK, LH_E_EMPTY, LH_E_BADARG, LH_E_HIP, LH_E_RCCL, LH_E_UNSUPPORTED, LH_E_STATE = range(7)
LH_ABI_VERSION = 5
LH_SOLVER_LDLT, LH_SOLVER_PCG = 0, 1
LH_PREC_FP64, LH_PREC_FP32_RESID = 0, 1
LH_COMM_RCCL, LH_COMM_HOST, LH_COMM_P2P = 0, 1, 2

# lh_allreduce_fn: int (*)(void* user, double* buf, int64_t count, int32_t op)   (op 0 sum, 1 max)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int64, C.c_int32)


class LhOptions(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("max_iters", C.c_int32), ("max_trials", C.c_int32),
        ("strategy", C.c_int32), ("huber_delta", C.c_double), ("stop_dchi2", C.c_double),
        ("tau", C.c_double), ("lambda_cap", C.c_double), ("lambda_init", C.c_double),
        ("linear_solver", C.c_int32), ("verbose", C.c_int32), ("device", C.c_int32),
        ("world_size", C.c_int32), ("rank", C.c_int32), ("degenerate_guard", C.c_int32),
        ("trials_per_sync", C.c_int32), ("profile", C.c_int32), ("pcg_max_iters", C.c_int32),
        ("pcg_tol", C.c_double), ("comm_id", C.c_uint8 * 128),
        ("gate_mode", C.c_int32), ("chunk_landmarks", C.c_int32), ("comm_mode", C.c_int32),
        ("host_threads", C.c_int32), ("allreduce", C.c_void_p), ("allreduce_user", C.c_void_p),
        ("precision", C.c_int32),
    ]


class LhWindow(C.Structure):
    _fields_ = [
        ("n_poses", C.c_int32), ("pose_Tcw", C.c_void_p), ("pose_fixed", C.c_void_p),
        ("n_landmarks", C.c_int32), ("lm_xyz", C.c_void_p),
        ("n_obs", C.c_int64), ("obs_pose", C.c_void_p), ("obs_lm", C.c_void_p),
        ("obs_cam", C.c_void_p), ("obs_uv", C.c_void_p),
        ("K", C.c_double * 4), ("n_cams", C.c_int32), ("cam_ext", C.c_void_p),
    ]


class LhResult(C.Structure):
    _fields_ = [
        ("pose_Tcw", C.c_void_p), ("lm_xyz", C.c_void_p), ("edge_robust_chi2", C.c_void_p),
        ("trace_chi2", C.c_void_p), ("trace_lambda", C.c_void_p), ("trace_cap", C.c_int32),
        ("trace_len", C.c_int32), ("iterations", C.c_int32), ("trials", C.c_int32),
        ("accepted", C.c_int32), ("chi2_initial", C.c_double), ("chi2_final", C.c_double),
        ("lambda_final", C.c_double), ("time_ms", C.c_double), ("pcg_iterations", C.c_int32),
        ("degenerate", C.c_int32), ("time_prep_ms", C.c_double), ("time_upload_ms", C.c_double),
        ("time_download_ms", C.c_double),
        # ABI 5: Backend::Optimize's outlier pass on the device (backend_lego.cpp:163-194)
        ("is_outlier", C.c_void_p), ("outlier_chi2_th", C.c_double), ("outlier_th", C.c_double),
        ("n_inlier", C.c_int64), ("n_outlier", C.c_int64),
    ]


class LhFrames(C.Structure):
    _fields_ = [
        ("n_frames", C.c_int32), ("obs_ptr", C.c_void_p), ("pose_Tcw", C.c_void_p), ("pts_w", C.c_void_p),
        ("obs_uv", C.c_void_p), ("is_outlier", C.c_void_p), ("K", C.c_double * 4),
    ]


class LhFramesResult(C.Structure):
    _fields_ = [
        ("pose_Tcw", C.c_void_p), ("is_outlier", C.c_void_p), ("edge_chi2", C.c_void_p),
        ("n_inliers", C.c_void_p), ("iterations", C.c_void_p), ("time_ms", C.c_double),
    ]


class LhLkInput(C.Structure):
    _fields_ = [
        ("cols", C.c_int32), ("rows", C.c_int32), ("step", C.c_int64), ("img1", C.c_void_p), ("img2", C.c_void_p),
        ("n_points", C.c_int32), ("kp1", C.c_void_p), ("inverse", C.c_int32), ("has_initial", C.c_int32),
        ("levels", C.c_int32),
    ]


class LhLkResult(C.Structure):
    _fields_ = [("kp2", C.c_void_p), ("success", C.c_void_p), ("time_ms", C.c_double)]


class LhKernelStats(C.Structure):
    _fields_ = [("launches", C.c_int64 * 8), ("total_ms", C.c_double * 8)]


# every symbol include/lego_ba.h declares (tests check the .so exports them all)
ABI_SYMBOLS = [
    "lh_strerror", "lh_default_options", "lh_default_options_v", "lh_kernel_name", "lh_comm_unique_id",
    "lh_create", "lh_destroy", "lh_solve", "lh_upload", "lh_solve_resident",
    "lh_kernel_stats_get", "lh_kernel_stats_reset", "lh_classify_outliers", "lh_set_profiling",
    "lh_estimate_pose", "lh_lk_track",
    "lh_debug_mfma_probe", "lh_debug_ldlt_probe", "lh_debug_pcg_probe", "lh_debug_event_floor", "lh_debug_stamps",
    "lh_debug_time_lin", "lh_debug_comm_count", "lh_debug_controller", "lh_debug_chains", "lh_debug_ladder",
    "lh_debug_batch",
]

_balib = None


def ba_lib():
    """Load liblego_ba.so.  Raises if it is missing: there is no fallback."""
    global _balib
    if _balib is None:
        if not os.path.exists(BA_LIB):
            raise RuntimeError(f"{BA_LIB} not built: the HIP extension is required (no CPU fallback)")
        lib = C.CDLL(BA_LIB)
        lib.lh_strerror.restype = C.c_char_p
        lib.lh_strerror.argtypes = [C.c_int]
        lib.lh_default_options.argtypes = [C.POINTER(LhOptions)]
        lib.lh_default_options_v.argtypes = [C.POINTER(LhOptions), C.c_int]
        lib.lh_kernel_name.restype = C.c_char_p
        lib.lh_kernel_name.argtypes = [C.c_int]
        lib.lh_comm_unique_id.argtypes = [C.c_void_p]
        lib.lh_create.argtypes = [C.POINTER(C.c_void_p), C.POINTER(LhOptions)]
        lib.lh_destroy.argtypes = [C.c_void_p]
        lib.lh_solve.argtypes = [C.c_void_p, C.POINTER(LhWindow), C.POINTER(LhResult)]
        lib.lh_upload.argtypes = [C.c_void_p, C.POINTER(LhWindow)]
        lib.lh_solve_resident.argtypes = [C.c_void_p, C.POINTER(LhResult)]
        lib.lh_kernel_stats_get.argtypes = [C.c_void_p, C.POINTER(LhKernelStats)]
        lib.lh_kernel_stats_reset.argtypes = [C.c_void_p]
        lib.lh_set_profiling.argtypes = [C.c_void_p, C.c_int]
        lib.lh_estimate_pose.argtypes = [C.c_void_p, C.POINTER(LhFrames), C.POINTER(LhFramesResult)]
        lib.lh_lk_track.argtypes = [C.c_void_p, C.POINTER(LhLkInput), C.POINTER(LhLkResult)]
        lib.lh_classify_outliers.argtypes = [C.c_void_p, C.c_int64, C.c_double, C.c_void_p,
                                             C.c_void_p, C.c_void_p, C.c_void_p]
        lib.lh_debug_event_floor.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
        lib.lh_debug_time_lin.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double)]
        lib.lh_debug_comm_count.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
        lib.lh_debug_controller.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
        lib.lh_debug_chains.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
        lib.lh_debug_ladder.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        if hasattr(lib, "lh_debug_batch"):   # (an older library of an A/B run lacks it)
            lib.lh_debug_batch.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        _balib = lib
    return _balib


def default_options(**kw):
    o = LhOptions()
    ba_lib().lh_default_options_v(C.byref(o), LH_ABI_VERSION)   # what the header's lh_default_options(&o) expands to
    for k, v in kw.items():
        if k == "comm_id":
            for i in range(128):
                o.comm_id[i] = v[i]
        else:
            setattr(o, k, v)
    return o


class LhError(RuntimeError):
    def __init__(self, status, where):
        self.status = status
        msg = ba_lib().lh_strerror(status).decode()
        super().__init__(f"{where}: {msg} ({status})")


def _check(st, where):
    if st != LH_OK:
        raise LhError(st, where)


def _as(a, dt):
    return None if a is None else np.ascontiguousarray(a, dtype=dt)


class _WindowRef:
    """Keeps the numpy arrays an LhWindow points to alive."""

    def __init__(self, w):
        self.arrays = dict(
            pose=_as(w["pose_Tcw"], np.float64), fixed=_as(w.get("pose_fixed"), np.uint8),
            lm=_as(w["lm_xyz"], np.float64), op=_as(w["obs_pose"], np.uint32),
            ol=_as(w["obs_lm"], np.uint32), oc=_as(w.get("obs_cam"), np.uint8),
            uv=_as(w["obs_uv"], np.float64), ext=_as(w.get("cam_ext"), np.float64),
        )
        a = self.arrays
        s = LhWindow()
        s.n_poses = a["pose"].shape[0]
        s.pose_Tcw = _ptr(a["pose"])
        s.pose_fixed = _ptr(a["fixed"])
        s.n_landmarks = a["lm"].shape[0]
        s.lm_xyz = _ptr(a["lm"])
        s.n_obs = a["op"].shape[0]
        s.obs_pose, s.obs_lm, s.obs_cam, s.obs_uv = _ptr(a["op"]), _ptr(a["ol"]), _ptr(a["oc"]), _ptr(a["uv"])
        for i in range(4):
            s.K[i] = float(w["K"][i])
        s.n_cams = 0 if a["ext"] is None else a["ext"].shape[0]
        s.cam_ext = _ptr(a["ext"])
        self.s = s


class Solver:
    """One lh_handle (one GPU / one landmark shard)."""

    def __init__(self, allreduce=None, **opts):
        """allreduce: optional Python callable f(buf: np.ndarray, op: int) reducing buf in place over
        the ranks (op 0 sum, 1 max), used with comm_mode=LH_COMM_HOST (the exchange) or LH_COMM_P2P (its bootstrap)
        and world_size > 1."""
        lib = ba_lib()
        self._cb = None
        if allreduce is not None:
            def _thunk(user, buf, count, op):
                try:
                    allreduce(np.ctypeslib.as_array(buf, shape=(count,)), int(op))
                    return 0
                except Exception:   # noqa: BLE001 - reported to the library as a failed exchange
                    return 1
            self._cb = ALLREDUCE_FN(_thunk)
            opts.setdefault("comm_mode", LH_COMM_HOST)
        self.opts = default_options(**opts)
        if self._cb is not None:
            self.opts.allreduce = C.cast(self._cb, C.c_void_p)
        h = C.c_void_p()
        _check(lib.lh_create(C.byref(h), C.byref(self.opts)), "lh_create")
        self.h = h
        self._win = None

    def close(self):
        if self.h:
            ba_lib().lh_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _result(self, n_poses, n_lm, n_obs, trace_cap=64, want_states=True, want_edges=True, reuse=None,
                outlier_chi2_th=None):
        def buf(key, shape, want):
            if not want:
                return None
            if reuse is not None and reuse.get(key) is not None and reuse[key].shape == shape:
                return reuse[key]
            return np.zeros(shape)
        out = dict(
            pose_Tcw=buf("pose_Tcw", (n_poses, 12), want_states),
            lm_xyz=buf("lm_xyz", (n_lm, 3), want_states),
            edge_robust_chi2=buf("edge_robust_chi2", (n_obs,), want_edges),
            trace_chi2=np.zeros(trace_cap), trace_lambda=np.zeros(trace_cap),
        )
        r = LhResult()
        r.pose_Tcw, r.lm_xyz = _ptr(out["pose_Tcw"]), _ptr(out["lm_xyz"])
        r.edge_robust_chi2 = _ptr(out["edge_robust_chi2"])
        r.trace_chi2, r.trace_lambda = _ptr(out["trace_chi2"]), _ptr(out["trace_lambda"])
        r.trace_cap = trace_cap
        if outlier_chi2_th is not None:   # the device outlier pass (ABI 5): flags instead of per-edge chi2
            prev = reuse.get("is_outlier") if reuse is not None else None   # a bool view of uint8 0 / 1
            ok = prev is not None and prev.shape == (n_obs,) and prev.dtype in (np.bool_, np.uint8)
            out["is_outlier"] = prev.view(np.uint8) if ok else np.zeros(n_obs, np.uint8)
            r.is_outlier = _ptr(out["is_outlier"])
            r.outlier_chi2_th = float(outlier_chi2_th)
        return r, out

    @staticmethod
    def _finish(r, out):
        n = r.trace_len
        out["trace_chi2"] = out["trace_chi2"][:n]
        out["trace_lambda"] = out["trace_lambda"][:n]
        for f in ("iterations", "trials", "accepted", "chi2_initial", "chi2_final", "lambda_final", "time_ms",
                  "pcg_iterations", "degenerate", "time_prep_ms", "time_upload_ms", "time_download_ms"):
            out[f] = getattr(r, f)
        if "is_outlier" in out:
            out["is_outlier"] = out["is_outlier"].view(bool)   # the device writes 0 / 1: no copy
            out["outlier_th"], out["n_inlier"], out["n_outlier"] = r.outlier_th, r.n_inlier, r.n_outlier
        return out

    def solve(self, w, trace_cap=64, reuse=None, outlier_chi2_th=None, want_edges=True):
        """lh_solve on host buffers.  reuse: a previous call's result dict whose output arrays are
        written again (a caller's persistent buffers) instead of freshly allocated ones.
        outlier_chi2_th: also run Backend::Optimize's outlier pass on the device from that threshold
        (is_outlier, outlier_th, n_inlier, n_outlier); want_edges=False then skips the per-edge chi2."""
        ref = _WindowRef(w)
        r, out = self._result(ref.s.n_poses, ref.s.n_landmarks, ref.s.n_obs, trace_cap, want_edges=want_edges,
                              reuse=reuse, outlier_chi2_th=outlier_chi2_th)
        _check(ba_lib().lh_solve(self.h, C.byref(ref.s), C.byref(r)), "lh_solve")
        return self._finish(r, out)

    def upload(self, w):
        self._win = _WindowRef(w)
        _check(ba_lib().lh_upload(self.h, C.byref(self._win.s)), "lh_upload")

    _SCALARS = ("iterations", "trials", "accepted", "chi2_initial", "chi2_final", "lambda_final", "time_ms",
                "pcg_iterations", "degenerate", "time_prep_ms", "time_upload_ms", "time_download_ms")

    def solve_resident(self, want_states=False, want_edges=False, trace_cap=64, outlier_chi2_th=None):
        if not want_states and not want_edges and outlier_chi2_th is None:
            # the array-free solve (the library's fast path): one lh_result and trace buffers per solver,
            # reused; the returned trace is a copy of the entries written
            fr = getattr(self, "_fast", None)
            if fr is None or fr[0] != trace_cap:
                tc, tl = np.zeros(trace_cap), np.zeros(trace_cap)
                r = LhResult()
                r.trace_chi2, r.trace_lambda, r.trace_cap = _ptr(tc), _ptr(tl), trace_cap
                fr = self._fast = (trace_cap, r, C.byref(r), tc, tl)
            _, r, rref, tc, tl = fr
            _check(ba_lib().lh_solve_resident(self.h, rref), "lh_solve_resident")
            n = r.trace_len
            out = {f: getattr(r, f) for f in self._SCALARS}
            out.update(pose_Tcw=None, lm_xyz=None, edge_robust_chi2=None, trace_chi2=tc[:n].copy(),
                       trace_lambda=tl[:n].copy())
            return out
        s = self._win.s
        r, out = self._result(s.n_poses, s.n_landmarks, s.n_obs, trace_cap, want_states, want_edges,
                              outlier_chi2_th=outlier_chi2_th)
        _check(ba_lib().lh_solve_resident(self.h, C.byref(r)), "lh_solve_resident")
        return self._finish(r, out)

    def lk_track(self, img1, img2, kp1, kp2_init=None, inverse=False, levels=4):
        """LKOpticalFlow4Layer (levels=4) / LKOpticalFlow1Layer (levels=1) of algorithm.cpp on 8-bit
        images (2-D uint8 arrays, rows contiguous).  Returns kp2 [n, 2] float32, success [n] bool and
        the device time."""
        i1 = np.ascontiguousarray(img1, dtype=np.uint8)
        i2 = np.ascontiguousarray(img2, dtype=np.uint8)
        if i1.shape != i2.shape or i1.ndim != 2:
            raise ValueError("images must be 2-D uint8 arrays of one shape")
        k1 = np.ascontiguousarray(kp1, dtype=np.float32).reshape(-1, 2)
        n = k1.shape[0]
        k2 = (np.zeros((n, 2), np.float32) if kp2_init is None
              else np.array(kp2_init, dtype=np.float32, copy=True).reshape(-1, 2))
        ok = np.zeros(n, np.uint8)
        a = LhLkInput()
        a.rows, a.cols = i1.shape
        a.step = i1.strides[0]
        a.img1, a.img2 = _ptr(i1), _ptr(i2)
        a.n_points, a.kp1 = n, _ptr(k1)
        a.inverse, a.has_initial, a.levels = int(bool(inverse)), int(kp2_init is not None), int(levels)
        r = LhLkResult()
        r.kp2, r.success = _ptr(k2), _ptr(ok)
        _check(ba_lib().lh_lk_track(self.h, C.byref(a), C.byref(r)), "lh_lk_track")
        return dict(kp2=k2, success=ok.astype(bool), time_ms=r.time_ms)

    def estimate_pose(self, fb, is_outlier_in=None):
        """Frontend::EstimateCurrentPose on every frame of batch `fb` (obs_ptr CSR, pose_Tcw, pts,
        obs_uv, K: the tests/frames.py layout) through lh_estimate_pose."""
        F = int(fb["n_frames"])
        keep = dict(ptr=_as(fb["obs_ptr"], np.int64), pose=_as(np.reshape(fb["pose_Tcw"], (F, 12)), np.float64),
                    pts=_as(fb["pts"], np.float64), uv=_as(fb["obs_uv"], np.float64),
                    fin=_as(is_outlier_in, np.uint8))
        O = int(keep["ptr"][-1]) if F else 0
        s = LhFrames()
        s.n_frames = F
        s.obs_ptr, s.pose_Tcw, s.pts_w, s.obs_uv = _ptr(keep["ptr"]), _ptr(keep["pose"]), _ptr(keep["pts"]), _ptr(keep["uv"])
        s.is_outlier = _ptr(keep["fin"])
        for i in range(4):
            s.K[i] = float(fb["K"][i])
        out = dict(pose_Tcw=np.zeros((F, 12)), is_outlier=np.zeros(O, np.uint8), edge_chi2=np.zeros(O),
                   n_inliers=np.zeros(F, np.int32), iterations=np.zeros(F, np.int32))
        r = LhFramesResult()
        r.pose_Tcw, r.is_outlier, r.edge_chi2 = _ptr(out["pose_Tcw"]), _ptr(out["is_outlier"]), _ptr(out["edge_chi2"])
        r.n_inliers, r.iterations = _ptr(out["n_inliers"]), _ptr(out["iterations"])
        _check(ba_lib().lh_estimate_pose(self.h, C.byref(s), C.byref(r)), "lh_estimate_pose")
        out["is_outlier"] = out["is_outlier"].astype(bool)
        out["time_ms"] = r.time_ms
        return out

    def kernel_stats(self):
        st = LhKernelStats()
        _check(ba_lib().lh_kernel_stats_get(self.h, C.byref(st)), "lh_kernel_stats_get")
        names = [ba_lib().lh_kernel_name(i).decode() for i in range(8)]
        return {names[i]: (st.launches[i], st.total_ms[i]) for i in range(8) if st.launches[i] > 0}

    def kernel_stats_reset(self):
        ba_lib().lh_kernel_stats_reset(self.h)

    def set_profiling(self, on):
        _check(ba_lib().lh_set_profiling(self.h, int(on)), "lh_set_profiling")

    def event_floor_ms(self):
        """HIP-event bracket of an empty kernel on this solver's stream (lh_debug_event_floor)."""
        ms = C.c_double(0.0)
        _check(ba_lib().lh_debug_event_floor(self.h, C.byref(ms)), "lh_debug_event_floor")
        return ms.value

    def time_lin_ms(self, reps=50):
        """k_lin's duration per LM trial (lh_debug_time_lin): replayed back to back after a solve."""
        ms = C.c_double(0.0)
        _check(ba_lib().lh_debug_time_lin(self.h, reps, C.byref(ms)), "lh_debug_time_lin")
        return ms.value

    def controller(self):
        """The controller the uploaded window runs (lh_debug_controller): 'k_ctrl', 'k_ctrl_g', 'k_ctrl_p'
        or 'k_ctrl_b'."""
        v = C.c_int(0)
        _check(ba_lib().lh_debug_controller(self.h, C.byref(v)), "lh_debug_controller")
        return ("k_ctrl", "k_ctrl_g", "k_ctrl_p", "k_ctrl_b")[v.value & 0xff]

    def band_loader_units(self):
        """k_ctrl_b's stream loaders take work units (some step needs more than 11; lh_debug_controller bit 9)."""
        v = C.c_int(0)
        _check(ba_lib().lh_debug_controller(self.h, C.byref(v)), "lh_debug_controller")
        return bool(v.value >> 9 & 1)

    def band_narrow(self):
        """k_ctrl_b runs its one-row-per-lane back substitution (every row's envelope within 56 rows of its
        8-row block; lh_debug_controller bit 8)."""
        v = C.c_int(0)
        _check(ba_lib().lh_debug_controller(self.h, C.byref(v)), "lh_debug_controller")
        return bool(v.value >> 8 & 1)

    def chains(self):
        """LM chains the last solve decided past the initial linearisation: its trials plus the
        re-linearisations of evaluate-only acceptances (lh_debug_chains)."""
        v = C.c_int(0)
        _check(ba_lib().lh_debug_chains(self.h, C.byref(v)), "lh_debug_chains")
        return v.value

    def ladder(self):
        """(rungs the uploaded window's factoring controller builds, rejections of the last solve that used a
        built rung instead of a factor) (lh_debug_ladder)."""
        r, k = C.c_int(0), C.c_int(0)
        _check(ba_lib().lh_debug_ladder(self.h, C.byref(r), C.byref(k)), "lh_debug_ladder")
        return r.value, k.value

    def batch(self):
        """(most rungs one chain of the uploaded window evaluates -- 1: batching off --, batches of evaluate-only
        rungs the last solve decided) (lh_debug_batch)."""
        return self.batch_detail()[:2]

    def batch_detail(self):
        """batch() and the acceptances inside the batches: (re-run as a full trial, re-run and stopping the loop)."""
        m, k, rt = C.c_int(0), C.c_int(0), (C.c_int * 2)()
        _check(ba_lib().lh_debug_batch(self.h, C.byref(m), C.byref(k), rt), "lh_debug_batch")
        return m.value, k.value, (rt[0], rt[1])

    def comm_count(self):
        """Reduced-system all-reduces the last solve issued (lh_debug_comm_count)."""
        n = C.c_int64(0)
        _check(ba_lib().lh_debug_comm_count(self.h, C.byref(n)), "lh_debug_comm_count")
        return n.value


def debug_stamps(reset=True):
    """Per-phase wave-cycle totals from the LH_STAMPS diagnostic build (zeros otherwise)."""
    lib = ba_lib()
    lib.lh_debug_stamps.argtypes = [C.c_void_p, C.c_int, C.c_int]
    out = (C.c_ulonglong * 256)()
    _check(lib.lh_debug_stamps(out, 256, int(reset)), "lh_debug_stamps")
    return np.array(out[:], dtype=np.uint64)


def comm_unique_id():
    buf = (C.c_uint8 * 128)()
    _check(ba_lib().lh_comm_unique_id(buf), "lh_comm_unique_id")
    return bytes(buf)


def classify_outliers(edge_rchi2, chi2_th=5.991):
    e = np.ascontiguousarray(edge_rchi2, np.float64)
    flags = np.zeros(e.shape[0], np.uint8)
    th, ni, no = C.c_double(), C.c_int64(), C.c_int64()
    _check(ba_lib().lh_classify_outliers(_ptr(e), e.shape[0], chi2_th, _ptr(flags), C.byref(th),
                                         C.byref(ni), C.byref(no)), "lh_classify_outliers")
    return flags.astype(bool), th.value, ni.value, no.value


# --------------------------------------------------------------------------
# window planner (liblego_plan.so: lh_plan.cpp alone, host C++; CPU tests and timings)
# --------------------------------------------------------------------------
PLAN_LIB = os.environ.get("LH_PLAN_LIB") or os.path.join(LIB_DIR, "liblego_plan.so")   # (env: sanitizer builds)
LH_TMAX = 6

# lh_chunk / lh_subbatch (lego-slam_amd/csrc/lh_common.h)
CHUNK_DT = np.dtype([("sb_begin", "<u4"), ("sb_end", "<u4"), ("U", "u1"), ("T", "u1"), ("pad", "u1", 2),
                     ("pose", "<u2", 16), ("item_base", "<u4")])
SUBBATCH_DT = np.dtype([("lm_begin", "<u4"), ("n_lm", "u1"), ("lg", "u1"), ("pad", "<u2")])

_planlib = None


def _pl():
    global _planlib
    if _planlib is None:
        if not os.path.exists(PLAN_LIB):
            raise RuntimeError(f"{PLAN_LIB} not built (run __graft_entry__.build())")
        lib = C.CDLL(PLAN_LIB)
        vp = C.c_void_p
        lib.lhp_plan_sizes.argtypes = [C.POINTER(LhWindow), C.c_int, C.c_int, vp, vp, C.c_int]
        lib.lhp_plan_fill.argtypes = [C.POINTER(LhWindow), C.c_int, C.c_int] + [vp] * 11 + [C.c_int]
        lib.lhp_plan_time.argtypes = [C.POINTER(LhWindow), C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double),
                                      C.POINTER(C.c_double)]
        if hasattr(lib, "lhp_plan_stages"):   # diagnostic entry point
            lib.lhp_plan_stages.argtypes = [C.POINTER(LhWindow), C.c_int, C.c_int, vp]
        lib.lhp_pool_stress.argtypes = [C.c_int, C.c_int, C.c_int]
        lib.lhp_ctrl_units.argtypes = [C.c_int, vp, C.c_int, vp]
        lib.lhp_ctrl_nd.argtypes = [C.c_int, vp, vp, vp, vp]
        lib.lhp_pool_stress.restype = C.c_int64
        _planlib = lib
    return _planlib


def plan_window(w, chunk_lm=0, threads=1, rank_invariant=False):
    """The device layout lh_upload builds for window `w` (lh_plan.cpp), as numpy arrays.  rank_invariant:
    the block list of a landmark-sharded handle (world_size > 1) past 64 poses."""
    ref = _WindowRef(w)
    sizes = np.zeros(7, np.int64)
    tg = np.zeros(LH_TMAX + 2, np.int32)
    _check(_pl().lhp_plan_sizes(C.byref(ref.s), chunk_lm, threads, _ptr(sizes), _ptr(tg), int(rank_invariant)),
           "lhp_plan_sizes")
    n_chunks, n_sb, n_items, npairs, n_rec, n_slots, fixed_mask = (int(x) for x in sizes)
    out = dict(chunks=np.zeros(n_chunks, CHUNK_DT), sbs=np.zeros(n_sb, SUBBATCH_DT),
               meta=np.zeros(n_slots, np.uint32), uv=np.zeros((n_slots, 2), np.float32), obs_perm=np.zeros(n_slots, np.int32),
               lm_perm=np.zeros(n_rec, np.int32), pair_ptr=np.zeros(npairs + 1, np.uint32),
               items=np.zeros(n_items, np.uint32), pair_pq=np.zeros((npairs, 2), np.uint16),
               rsmap=np.zeros(npairs * 36, np.uint32), lm_xyz=np.zeros((ref.s.n_landmarks, 3)))
    k = ("chunks", "sbs", "meta", "uv", "obs_perm", "lm_perm", "pair_ptr", "items", "pair_pq", "rsmap", "lm_xyz")
    _check(_pl().lhp_plan_fill(C.byref(ref.s), chunk_lm, threads, *[_ptr(out[n]) for n in k], int(rank_invariant)),
           "lhp_plan_fill")
    out.update(tgroup_begin=tg, fixed_mask=fixed_mask)
    return out


def ctrl_units(n, fcb, band=False):
    """The controllers' per-step work-unit table (lh_ctrl_units) for an n-row reduced system whose tile row
    I first reaches 8-column block fcb[I]: (units[16 waves][steps] as uint16, most units a step needed)."""
    steps = 6 * 256 // 8 if band else 16
    f = np.ascontiguousarray(fcb, np.int32)
    u = np.zeros(16 * steps, np.uint16)
    worst = _pl().lhp_ctrl_units(int(n), _ptr(f), int(bool(band)), _ptr(u))
    return u.reshape(16, steps), worst


def ctrl_nd(pf):
    """k_ctrl's two-chain schedule (lh_ctrl_nd_plan) for a window whose pose p first couples pose pf[p]:
    dict(nsteps, a, s, long_first, units[16][16] uint16, pos[P]); nsteps 0 = no split."""
    P = len(pf)
    f = np.ascontiguousarray(pf, np.int32)
    info = np.zeros(4, np.int32)
    u = np.zeros(16 * 16, np.uint16)
    pos = np.zeros(max(P, 1), np.uint8)
    _pl().lhp_ctrl_nd(int(P), _ptr(f), _ptr(info), _ptr(u), _ptr(pos))
    return {"nsteps": int(info[0]), "a": int(info[1]), "s": int(info[2]), "long_first": int(info[3]),
            "units": u.reshape(16, 16), "pos": pos[:P].astype(np.int64)}


def pool_stress(threads, runs, n):
    """Sum of every index the planner's worker pool visits over `runs` back-to-back jobs of size n."""
    return int(_pl().lhp_pool_stress(threads, runs, n))


def plan_stages_ms(w, threads=1, reps=3):
    """Diagnostic: plan_structure's stage end times in ms (index checks, CSR, per-landmark sort and
    masks, span order, chunking, sub-batches, reduce-plan sizes)."""
    ref = _WindowRef(w)
    out = np.zeros(7)
    _check(_pl().lhp_plan_stages(C.byref(ref.s), threads, reps, _ptr(out)), "lhp_plan_stages")
    return out


def plan_time_ms(w, chunk_lm=0, threads=1, reps=5):
    """Host preprocessing time of lh_upload for window `w`: (plan_structure ms, plan_fill ms)."""
    ref = _WindowRef(w)
    a, b = C.c_double(), C.c_double()
    _check(_pl().lhp_plan_time(C.byref(ref.s), chunk_lm, threads, reps, C.byref(a), C.byref(b)), "lhp_plan_time")
    return a.value, b.value

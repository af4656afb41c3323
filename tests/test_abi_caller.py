"""The drop-in boundary from C++: tests/abi_caller.cpp is the INTEGRATION.md section 3 flow
(Backend::Optimize around the solver: lh_create, lh_solve, lh_classify_outliers, write-back values,
src/backend_lego.cpp:56-218) compiled against include/lego_ba.h and linked to liblego_ba.so with no
Python in between.  CPU: it compiles and links from source.  GPU: the prebuilt caller
(lego-slam_amd/lib/abi_caller, built by `make`) solves a golden window and its outputs match the
fixture (oracle) values."""
import glob
import os
import subprocess

import numpy as np
import pytest

import lego_ba

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "abi_caller.cpp")
EXE = os.path.join(ROOT, "lego-slam_amd", "lib", "abi_caller")


def write_window(path, w):
    P, L, O = len(w["pose_Tcw"]), len(w["lm_xyz"]), len(w["obs_pose"])
    ext = w.get("cam_ext")
    ncam = 0 if ext is None else len(ext)
    fixed = w.get("pose_fixed")
    with open(path, "wb") as f:
        np.array([P, L], np.int32).tofile(f)
        np.array([O], np.int64).tofile(f)
        np.array([ncam, 0 if fixed is None else 1], np.int32).tofile(f)
        np.asarray(w["K"], np.float64).tofile(f)
        np.asarray(w["pose_Tcw"], np.float64).tofile(f)
        if fixed is not None:
            np.asarray(fixed, np.uint8).tofile(f)
        np.asarray(w["lm_xyz"], np.float64).tofile(f)
        np.asarray(w["obs_pose"], np.uint32).tofile(f)
        np.asarray(w["obs_lm"], np.uint32).tofile(f)
        np.asarray(w["obs_cam"] if w.get("obs_cam") is not None else np.zeros(O), np.uint8).tofile(f)
        np.asarray(w["obs_uv"], np.float64).tofile(f)
        if ncam:
            np.asarray(ext, np.float64).tofile(f)


def read_result(path, P, L, O):
    b = open(path, "rb").read()
    off = 0

    def take(dt, n):
        nonlocal off
        a = np.frombuffer(b, dt, n, off)
        off += a.nbytes
        return a
    st, it, tr, acc = take(np.int32, 4)
    chi0, chi, th = take(np.float64, 3)
    nin, nout = take(np.int64, 2)
    return dict(status=int(st), iterations=int(it), trials=int(tr), accepted=int(acc), chi2_initial=chi0,
                chi2_final=chi, chi2_th=th, n_inlier=int(nin), n_outlier=int(nout),
                pose_Tcw=take(np.float64, 12 * P).reshape(P, 12), lm_xyz=take(np.float64, 3 * L).reshape(L, 3),
                edge_robust_chi2=take(np.float64, O), is_outlier=take(np.uint8, O).astype(bool))


def test_caller_compiles_and_links_from_source(tmp_path):
    exe = tmp_path / "abi_caller"
    lib_dir = os.path.dirname(lego_ba.BA_LIB)
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), SRC,
                           "-o", str(exe), "-L", lib_dir, "-llego_ba", f"-Wl,-rpath,{lib_dir}"])
    out = subprocess.run(["ldd", str(exe)], capture_output=True, text=True).stdout
    assert "liblego_ba.so" in out and "not found" not in out.split("liblego_ba.so")[1].splitlines()[0]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1_stable_noout_s0", "mini_stable_noout_s0"])
def test_caller_solves_golden_window(tmp_path, name):
    z = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
    w = {k[3:]: z[k] for k in z.files if k.startswith("in_")}
    win, res = tmp_path / "w.bin", tmp_path / "r.bin"
    write_window(win, w)
    subprocess.run([EXE, str(win), str(res)], check=True, timeout=120)
    r = read_result(res, len(w["pose_Tcw"]), len(w["lm_xyz"]), len(w["obs_pose"]))
    assert r["status"] == 0
    assert r["iterations"] == int(z["out_iterations"]) and r["trials"] == int(z["out_trials"])
    assert abs(r["chi2_final"] - float(z["out_chi2_final"])) < 1e-6 * float(z["out_chi2_final"])
    assert np.allclose(r["pose_Tcw"], z["out_pose_Tcw"], atol=1e-6)
    assert np.allclose(r["lm_xyz"], z["out_lm_xyz"], atol=1e-6)
    flags, th, ni, no = lego_ba.classify_outliers(z["out_edge_robust_chi2"])
    assert r["chi2_th"] == th and np.mean(r["is_outlier"] != flags) < 1e-3

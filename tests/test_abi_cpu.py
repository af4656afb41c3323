"""CPU tests of the C-ABI boundary (include/lego_ba.h): the shared library
loads and exports every declared symbol, the ctypes structs match the C
layout, option defaults mirror the reference constants, and the host-only
Backend::Optimize outlier pass (backend_lego.cpp:163-194) is exact.
No compute call is made here (no GPU in this container)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import lego_ba

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "lego_ba.h")


def declared_functions():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(lh_\w+)\s*\(", txt, re.M)))


def test_library_loads_and_exports_every_header_symbol():
    lib = lego_ba.ba_lib()
    decl = declared_functions()
    assert len(decl) >= 12
    assert set(lego_ba.ABI_SYMBOLS) <= set(decl)
    for name in decl:
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", lego_ba.BA_LIB], capture_output=True, text=True).stdout
    for name in decl:
        assert re.search(rf"\bT {name}\b", out), name


def test_no_hipify_or_dual_paths_in_sources():
    src = os.path.join(ROOT, "lego-slam_amd", "csrc")
    for f in os.listdir(src):
        txt = open(os.path.join(src, f)).read()
        assert "__HIP_PLATFORM_AMD__" not in txt and "cuda" not in txt.lower(), f


LAYOUT_C = r"""
#include <stddef.h>
#include <stdio.h>
#include "lego_ba.h"
#define P(s, f) printf(#s "." #f " %zu\n", offsetof(s, f));
int main(void) {
  printf("lh_options %zu\n", sizeof(lh_options));
  printf("lh_window %zu\n", sizeof(lh_window));
  printf("lh_result %zu\n", sizeof(lh_result));
  printf("lh_kernel_stats %zu\n", sizeof(lh_kernel_stats));
  printf("lh_frames %zu\n", sizeof(lh_frames));
  printf("lh_frames_result %zu\n", sizeof(lh_frames_result));
  P(lh_frames, obs_ptr) P(lh_frames, is_outlier) P(lh_frames, K)
  P(lh_frames_result, iterations) P(lh_frames_result, time_ms)
  P(lh_options, huber_delta) P(lh_options, linear_solver) P(lh_options, comm_id) P(lh_options, profile)
  P(lh_options, pcg_max_iters) P(lh_options, pcg_tol)
  P(lh_options, gate_mode) P(lh_options, chunk_landmarks) P(lh_options, comm_mode) P(lh_options, host_threads)
  P(lh_options, allreduce) P(lh_options, allreduce_user) P(lh_options, precision)
  P(lh_window, n_obs) P(lh_window, K) P(lh_window, cam_ext)
  P(lh_result, trace_cap) P(lh_result, chi2_initial) P(lh_result, time_ms) P(lh_result, pcg_iterations)
  P(lh_result, degenerate) P(lh_result, time_prep_ms) P(lh_result, time_upload_ms) P(lh_result, time_download_ms)
  P(lh_result, is_outlier) P(lh_result, outlier_chi2_th) P(lh_result, outlier_th) P(lh_result, n_inlier)
  P(lh_result, n_outlier)
  return 0;
}
"""


def test_ctypes_struct_layout_matches_header(tmp_path):
    c = tmp_path / "layout.c"
    c.write_text(LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)])
    got = dict(line.rsplit(" ", 1) for line in subprocess.check_output([str(exe)], text=True).splitlines())
    got = {k: int(v) for k, v in got.items()}
    assert got["lh_options"] == C.sizeof(lego_ba.LhOptions)
    assert got["lh_window"] == C.sizeof(lego_ba.LhWindow)
    assert got["lh_result"] == C.sizeof(lego_ba.LhResult)
    assert got["lh_kernel_stats"] == C.sizeof(lego_ba.LhKernelStats)
    assert got["lh_frames"] == C.sizeof(lego_ba.LhFrames)
    assert got["lh_frames_result"] == C.sizeof(lego_ba.LhFramesResult)
    for key, v in got.items():
        if "." in key:
            s, f = key.split(".")
            cls = {"lh_options": lego_ba.LhOptions, "lh_window": lego_ba.LhWindow, "lh_result": lego_ba.LhResult,
                   "lh_frames": lego_ba.LhFrames, "lh_frames_result": lego_ba.LhFramesResult}[s]
            assert getattr(cls, f).offset == v, key


def test_default_options_are_keyed_on_the_callers_abi():
    """A binary built against the ABI-4 header calls the plain symbol lh_default_options: it gets abi_version 4, so
    the library never reads the ABI-5 lh_result fields its smaller struct lacks.  The header maps
    lh_default_options(&o) to lh_default_options_v(&o, LH_ABI_VERSION), the caller's compile-time version."""
    lib = lego_ba.ba_lib()
    o = lego_ba.LhOptions()
    o.abi_version = 99
    lib.lh_default_options(C.byref(o))
    assert o.abi_version == 4 and o.max_iters == 10 and o.huber_delta == 5.991
    lib.lh_default_options_v(C.byref(o), 5)
    assert o.abi_version == 5 and o.max_iters == 10
    hdr = open(os.path.join(ROOT, "include", "lego_ba.h")).read()
    assert "#define lh_default_options(opt) lh_default_options_v((opt), LH_ABI_VERSION)" in hdr


def test_default_options_mirror_reference_constants():
    o = lego_ba.default_options()
    assert o.abi_version == lego_ba.LH_ABI_VERSION == 5
    assert o.precision == lego_ba.LH_PREC_FP64          # double throughout: the residual mirrors the reference
    assert o.gate_mode == 0 and o.degenerate_guard == 0   # the reference's Huber gate and LU semantics
    assert o.comm_mode == lego_ba.LH_COMM_RCCL and o.chunk_landmarks == 0 and not o.allreduce
    assert o.linear_solver == lego_ba.LH_SOLVER_LDLT   # Eigen LDLT     problem.cpp:420
    assert o.pcg_tol == 1e-6 and o.pcg_max_iters <= 0   # PCGSolver stop rule / cap  problem.cpp:597, :422
    assert o.max_iters == 10          # problem.solve(10)      backend_lego.cpp:161
    assert o.max_trials == 10         # false_cnt_threshold    problem.cpp:178
    assert o.huber_delta == 5.991     # HuberCost(chi2_th)     backend_lego.cpp:92-94
    assert o.stop_dchi2 == 1e-5       # diffChiThreshold_      problem.h:165
    assert o.tau == 1e-5 and o.lambda_cap == 5e10   # problem.cpp:494-495
    assert o.lambda_init < 0 and o.strategy == 0 and o.world_size == 1


def test_strerror():
    lib = lego_ba.ba_lib()
    for st in range(7):
        assert lib.lh_strerror(st)
    assert b"empty" in lib.lh_strerror(lego_ba.LH_E_EMPTY)


def reference_outlier_pass(rchi2, chi2_th):
    """Python transcription of backend_lego.cpp:163-194."""
    cnt_out = cnt_in = 0
    iteration = 0
    while iteration < 5:
        cnt_out = int(np.sum(rchi2 > chi2_th))
        cnt_in = len(rchi2) - cnt_out
        ratio = cnt_in / float(cnt_in + cnt_out) if (cnt_in + cnt_out) else float("nan")
        if ratio > 0.5:
            break
        chi2_th *= 2
        iteration += 1
    return rchi2 > chi2_th, chi2_th, cnt_in, cnt_out


@pytest.mark.parametrize("frac", [0.0, 0.3, 0.6, 0.9, 1.0])
def test_classify_outliers_matches_backend(frac):
    rng = np.random.default_rng(int(frac * 10))
    n = 1000
    r = rng.uniform(0, 5.0, n)
    m = rng.random(n) < frac
    r[m] = rng.uniform(6.0, 400.0, m.sum())
    flags, th, ni, no = lego_ba.classify_outliers(r)
    rf, rth, rni, rno = reference_outlier_pass(r, 5.991)
    assert np.array_equal(flags, rf) and th == rth and (ni, no) == (rni, rno)


def test_classify_outliers_empty():
    flags, th, ni, no = lego_ba.classify_outliers(np.zeros(0))
    assert th == 5.991 * 32 and ni == 0 and no == 0

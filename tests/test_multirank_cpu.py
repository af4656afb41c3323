"""The N>1 path on CPU (gloo, world_size 2): landmark shards, one all-reduce.

The multi-GPU solver shards landmarks across ranks, replicates poses, and
all-reduces the packed reduced pose system (S, bs, chi2 and gain-scale partials) once per LM
trial; every rank then runs the same deterministic solve.  This is correct iff the Schur
reduction is additive over landmark shards.  Here two gloo ranks each reduce their shard with
the oracle (oracle/lego_oracle.c orc_reduced_system), all-reduce, and must reproduce the
full-window system; and the sharded window generator (bench.py's per-rank input) must hand
each rank exactly its slice of the global window.
"""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import lego_ba
import oracle_bind as ob
from windows import window


def _rendezvous_file():
    # a file store: no TCP port to race for (a port probed free can be taken before the store binds it)
    fd, path = tempfile.mkstemp(prefix="lh_rdzv_")
    os.close(fd)
    os.unlink(path)
    return path


def _rank_main(rank, world, rdzv, cfg, seed, family, q):
    dist.init_process_group("gloo", init_method="file://" + rdzv, rank=rank, world_size=world)
    try:
        w = window(cfg, seed=seed, family=family)
        L = len(w["lm_xyz"])
        l0, l1 = rank * L // world, (rank + 1) * L // world
        S, bs, chi2 = ob.reduced_system(ob.landmark_shard(w, l0, l1), n_threads=1)
        buf = torch.from_numpy(np.concatenate([S.ravel(), bs, [chi2]]))
        dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        if rank == 0:
            q.put(buf.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg,seed,family", [("C1", 0, "default"), ("mini", 1, "stable")])
def test_landmark_shards_allreduce_to_full_reduced_system(cfg, seed, family):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    rdzv = _rendezvous_file()
    procs = [ctx.Process(target=_rank_main, args=(r, world, rdzv, cfg, seed, family, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=120)
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    finally:
        if os.path.exists(rdzv):
            os.unlink(rdzv)
    w = window(cfg, seed=seed, family=family)
    S, bs, chi2 = ob.reduced_system(w, n_threads=1)
    n = S.shape[0]
    Sg, bsg, chi2g = got[:n * n].reshape(n, n), got[n * n:n * n + n], got[-1]
    scale = np.abs(S).max()
    assert np.abs(Sg - S).max() <= 1e-12 * scale
    assert np.abs(bsg - bs).max() <= 1e-12 * np.abs(bs).max()
    assert abs(chi2g - chi2) <= 1e-12 * chi2


def test_sharded_window_generation_matches_global_window():
    """bench.py generates each rank's shard directly (lm_begin/lm_end): it must equal the
    global window restricted to that landmark range, poses identical on every rank."""
    P, L, k, seed = 10, 3000, 8, 5
    full = lego_ba.generate_window(P=P, L=L, k=k, seed=seed)
    for r in range(3):
        l0, l1 = r * L // 3, (r + 1) * L // 3
        part = lego_ba.generate_window(P=P, L=L, k=k, seed=seed, lm_begin=l0, lm_end=l1)
        ref = ob.landmark_shard(full, l0, l1)
        assert np.array_equal(part["pose_Tcw"], full["pose_Tcw"])
        assert np.array_equal(part["lm_xyz"], ref["lm_xyz"])
        order_p = np.lexsort((part["obs_pose"], part["obs_lm"]))
        order_r = np.lexsort((ref["obs_pose"], ref["obs_lm"]))
        for key in ("obs_pose", "obs_lm", "obs_uv"):
            assert np.array_equal(np.asarray(part[key])[order_p], np.asarray(ref[key])[order_r]), key


def test_bench_c4_strong_scaling_shards():
    """bench.py's N > 1 default is BASELINE config 4's C4 window at every N (strong scaling): rank r of N holds
    landmarks [L r / N, L (r + 1) / N) of the one window, the ranks' shards together are the window, and value
    counts C3-equivalent work (C4 = 10 C3 windows; C3w, the weak-scaling side workload, N).  (The shards are
    checked at a reduced size through the same make_window path.)"""
    import importlib
    import sys
    sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
    bench = importlib.import_module("bench")
    assert bench.default_workload(1) == "C3" and all(bench.default_workload(n) == "C4" for n in (2, 4, 8))
    assert bench.c3_units("C3", 1) == 1.0 and all(bench.c3_units("C4", n) == 10.0 for n in (1, 2, 8))
    assert bench.c3_units("C3w", 4) == 4.0
    c4 = bench.WORKLOADS["C4"]
    assert (c4["P"], c4["L"], c4["k"]) == (20, 500_000, 8)   # 4 000 000 observations
    saved = dict(bench.WORKLOADS)
    try:
        bench.WORKLOADS["C4"] = dict(P=8, L=1800, k=6)
        full = bench.make_window("C4", "stable_noout", 0, 0, 1)
        for n in (2, 3):
            parts = [bench.make_window("C4", "stable_noout", 0, r, n) for r in range(n)]
            assert sum(len(p["lm_xyz"]) for p in parts) == 1800
            assert np.array_equal(np.vstack([p["lm_xyz"] for p in parts]), full["lm_xyz"])
            assert np.array_equal(np.concatenate([p["obs_uv"] for p in parts]), full["obs_uv"])
            for r, p in enumerate(parts):
                ref = ob.landmark_shard(full, 1800 * r // n, 1800 * (r + 1) // n)
                assert np.array_equal(p["lm_xyz"], ref["lm_xyz"])
                assert np.array_equal(p["pose_Tcw"], full["pose_Tcw"]) and p["pose_fixed"][0] == 1
    finally:
        bench.WORKLOADS.clear()
        bench.WORKLOADS.update(saved)

"""The landmark-sharded multi-rank solve through the real solver (liblego_ba.so, HIP kernels), on the
one GPU of a test box: two processes, each with its own handle (world_size 2) and its landmark shard,
exchanging the packed reduced pose system once per LM trial over gloo through the ABI's host
transport (lh_options.comm_mode = LH_COMM_HOST; RCCL cannot pair two ranks on one device).  Every
device-side piece of the N-GPU path runs: shard upload, per-shard linearisation and Schur reduction,
the MAX exchange of max|diag H_ll| for lambda_0, the SUM exchange of S, b_s, b_p, chi2 and gain-scale
partials, and the identical per-rank controller.  The result must match the one-rank solve of the
whole window, and both ranks must hold bit-identical poses.  (the RCCL transport's
collective count is covered by test_gpu_parity.py::test_collective_count_is_a_function_of_the_stop_trial.)
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, cfg, seed, family, opts, q):
    import torch
    import torch.distributed as dist

    import lego_ba
    from windows import window

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def allreduce(buf, op):
            t = torch.from_numpy(buf)   # shares the library's host buffer
            dist.all_reduce(t, op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MAX)

        w = window(cfg, seed=seed, family=family)
        L = len(w["lm_xyz"])
        l0, l1 = rank * L // world, (rank + 1) * L // world
        keep = (w["obs_lm"] >= l0) & (w["obs_lm"] < l1)
        shard = dict(w, lm_xyz=w["lm_xyz"][l0:l1], obs_lm=(w["obs_lm"][keep] - l0).astype(np.uint32),
                     obs_pose=w["obs_pose"][keep], obs_cam=w["obs_cam"][keep], obs_uv=w["obs_uv"][keep])
        s = lego_ba.Solver(device=0, world_size=world, rank=rank, allreduce=allreduce, **opts)
        r = s.solve(shard)
        r["exchanges"] = s.comm_count()
        s.close()
        q.put((rank, {k: v for k, v in r.items()}))
    finally:
        dist.destroy_process_group()


def run_sharded(cfg, seed, family, world=2, **opts):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, cfg, seed, family, opts, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, r = q.get(timeout=100)
            out[rank] = r
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return out


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


@pytest.mark.parametrize("cfg,seed,family", [("C2", 0, "stable_noout"), ("mini", 2, "default"), ("W32", 1, "stable_noout")])
def test_two_rank_sharded_solve_matches_one_rank(cfg, seed, family):
    import lego_ba
    from windows import window
    w = window(cfg, seed=seed, family=family)
    one = lego_ba.Solver().solve(w)
    out = run_sharded(cfg, seed, family)
    a, b = out[0], out[1]
    # identical controller on both ranks: same trajectory, bit-identical poses
    assert (a["iterations"], a["trials"]) == (b["iterations"], b["trials"])
    assert a["chi2_final"] == b["chi2_final"] and np.array_equal(a["pose_Tcw"], b["pose_Tcw"])
    assert a["exchanges"] == b["exchanges"] == a["trials"] + 1
    # = the one-rank solve of the whole window, to summation order
    assert a["iterations"] == one["iterations"] and a["trials"] == one["trials"]
    assert rel(a["chi2_initial"], one["chi2_initial"]) < 1e-12
    assert rel(a["chi2_final"], one["chi2_final"]) < 1e-9
    L = len(w["lm_xyz"])
    lm = np.vstack([a["lm_xyz"], b["lm_xyz"]])
    assert lm.shape == (L, 3)
    if family.startswith("stable"):
        assert np.allclose(a["pose_Tcw"], one["pose_Tcw"], atol=1e-9)
        assert np.allclose(lm, one["lm_xyz"], atol=1e-7)
    else:
        # survey-default windows (gauge free, reference Huber gate): summation order moves the
        # states by as much as the oracle's own reorderings do (tests/align.py)
        from align import oracle_state_spread
        _, lm_sp, pose_sp = oracle_state_spread(w, threads=(1, 2, 8))
        assert np.abs(a["pose_Tcw"] - one["pose_Tcw"]).max() <= max(1e-5, 10 * pose_sp)
        assert np.abs(lm - one["lm_xyz"]).max() <= max(1e-5, 10 * lm_sp)
    rho = np.concatenate([a["edge_robust_chi2"], b["edge_robust_chi2"]])
    assert rel(rho.sum(), one["edge_robust_chi2"].sum()) < 1e-9

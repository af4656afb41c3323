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
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rendezvous_file():
    # a file store: no TCP port to race for (a port probed free can be taken by an outgoing
    # connection before the store binds it: EADDRINUSE was seen on a test box)
    fd, path = tempfile.mkstemp(prefix="lh_rdzv_")
    os.close(fd)
    os.unlink(path)
    return path


def _rank_main(rank, world, rdzv, cfg, seed, family, opts, q):
    import torch
    import torch.distributed as dist

    import lego_ba
    from windows import window_shard

    dist.init_process_group("gloo", init_method="file://" + rdzv, rank=rank, world_size=world)
    try:
        def allreduce(buf, op):
            t = torch.from_numpy(buf)   # shares the library's host buffer
            dist.all_reduce(t, op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MAX)

        os.environ.update(opts.pop("env", {}))
        corrupt = opts.pop("corrupt_rank", None)
        fail_after = opts.pop("fail_after_rank", None)
        if fail_after is not None:   # lh_host.cpp's test hook: that rank fails after the envelope collective
            os.environ["LH_TEST_FAIL_AFTER_ENVELOPE"] = str(fail_after)
        if isinstance(cfg, dict):   # a generated window (lego_ba.generate_window arguments), sharded by landmark
            L = cfg["L"]
            shard = sharded_generated(cfg, rank * L // world, (rank + 1) * L // world, seed)
        else:
            L = lego_ba.CONFIGS[cfg]["L"]
            shard = window_shard(cfg, rank * L // world, (rank + 1) * L // world, seed=seed, family=family)
        if corrupt == rank:   # a pixel no float holds: this rank's upload fails in the planner's fill
            shard["obs_uv"] = np.array(shard["obs_uv"], np.float64)
            shard["obs_uv"][len(shard["obs_uv"]) // 2, 0] = 100.1
        oth = opts.pop("outlier_th", None)
        s = lego_ba.Solver(device=0, world_size=world, rank=rank, allreduce=allreduce, **opts)
        try:
            r = s.solve(shard) if oth is None else s.solve(shard, outlier_chi2_th=oth)
        except lego_ba.LhError as e:
            q.put((rank, {"status": e.status}))
            s.close()
            return
        r["exchanges"] = s.comm_count()
        r["chains"] = s.chains()
        r["batch"] = s.batch()
        r["controller"] = s.controller()
        r["status"] = 0
        s.close()
        q.put((rank, {k: v for k, v in r.items()}))
    finally:
        dist.destroy_process_group()


def stable_generated(P, L, k=8, **kw):
    """Generator arguments of a sliding window of P keyframes (landmarks seen by runs of k consecutive
    keyframes), the stable family without outliers, first pose fixed: reproducible under reordering."""
    from windows import STABLE
    return dict(P=P, L=L, k=k, **dict(STABLE, outlier_frac=0.0), **kw)


def sharded_generated(spec, l0, l1, seed):
    import lego_ba
    w = lego_ba.generate_window(seed=seed, lm_begin=l0, lm_end=l1, **spec)
    f = np.zeros(spec["P"], np.uint8)
    f[0] = 1
    w["pose_fixed"] = f
    return w


def run_sharded(cfg, seed, family, world=2, timeout=100, **opts):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    rdzv = _rendezvous_file()
    procs = [ctx.Process(target=_rank_main, args=(r, world, rdzv, cfg, seed, family, opts, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, r = q.get(timeout=timeout)
            out[rank] = r
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        if os.path.exists(rdzv):
            os.unlink(rdzv)
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
    assert a["exchanges"] == b["exchanges"] == a["chains"] + 1 and a["chains"] + 15 * a["batch"][1] >= a["trials"]
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


# ---------------------------------------------------------------------------------------------
# C4 (BASELINE configs[3], the multi-GPU window: 20 KF / 500 k landmarks / 4 M observations) sharded
# 2 and 4 ways.  With the reference Huber gate (base_edge.cpp:55) the C4 trajectory is not
# reproducible even by the oracle under a change of summation order (test_gpu_parity.py::
# test_c4_window_one_gpu_parity), and sharding changes the summation order of S.  With the gate's
# rounding residue taken as 0 on both sides (gate_mode 1) the oracle reproduces to 1e-14 across
# thread counts, so the sharded solve is held to the north-star bar there: the oracle's iterations
# and trials, final chi2 1e-6, poses and landmarks 1e-6 — and to the one-rank solve of the whole
# window to summation order.  (problem.cpp:179-219: the LM loop every rank runs on identical sums.)
# ---------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def c4_gate1():
    import lego_ba
    import oracle_bind as ob
    from windows import window
    w = window("C4", seed=0, family="stable_noout")
    s = lego_ba.Solver(gate_mode=1)
    one = s.solve(w)
    s.close()
    o = ob.solve(w, n_threads=16, gate_mode=1)
    return w, one, o


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", [2, 4])
def test_c4_sharded_solve_matches_oracle_and_one_rank(c4_gate1, world):
    w, one, o = c4_gate1
    out = run_sharded("C4", 0, "stable_noout", world=world, timeout=400, gate_mode=1)
    a = out[0]
    for r in range(1, world):
        b = out[r]
        assert (a["iterations"], a["trials"], a["chi2_final"]) == (b["iterations"], b["trials"], b["chi2_final"])
        assert np.array_equal(a["pose_Tcw"], b["pose_Tcw"])
        assert np.array_equal(a["trace_chi2"], b["trace_chi2"]) and np.array_equal(a["trace_lambda"], b["trace_lambda"])
        assert b["exchanges"] == a["exchanges"] == a["chains"] + 1 and a["chains"] + 15 * a["batch"][1] >= a["trials"]
    lm = np.vstack([out[r]["lm_xyz"] for r in range(world)])
    rho = np.concatenate([out[r]["edge_robust_chi2"] for r in range(world)])
    assert lm.shape == w["lm_xyz"].shape
    # the oracle (north-star bar)
    assert (a["iterations"], a["trials"]) == (o["iterations"], o["trials"])
    assert rel(a["chi2_initial"], o["chi2_initial"]) < 1e-12
    assert rel(a["chi2_final"], o["chi2_final"]) < 1e-6
    assert np.allclose(a["trace_chi2"], o["trace_chi2"], rtol=1e-9)
    assert np.allclose(a["pose_Tcw"], o["pose_Tcw"], atol=1e-6)
    assert np.allclose(lm, o["lm_xyz"], atol=1e-6)
    # the one-rank solve of the whole window (same kernels, summation order only)
    assert (a["iterations"], a["trials"]) == (one["iterations"], one["trials"])
    assert rel(a["chi2_final"], one["chi2_final"]) < 1e-9
    assert np.allclose(a["trace_lambda"], one["trace_lambda"], rtol=1e-9)
    assert np.allclose(a["pose_Tcw"], one["pose_Tcw"], atol=1e-8)
    assert np.allclose(lm, one["lm_xyz"], atol=1e-7)
    assert rel(rho.sum(), one["edge_robust_chi2"].sum()) < 1e-9


def _create_main(rank, world, rdzv, opts_per_rank, q):
    import torch
    import torch.distributed as dist

    import lego_ba

    dist.init_process_group("gloo", init_method="file://" + rdzv, rank=rank, world_size=world)
    try:
        def allreduce(buf, op):
            t = torch.from_numpy(buf)
            dist.all_reduce(t, op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MAX)
        try:
            s = lego_ba.Solver(device=0, world_size=world, rank=rank, allreduce=allreduce, **opts_per_rank[rank])
            s.close()
            q.put((rank, 0))
        except lego_ba.LhError as e:
            q.put((rank, e.status))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("opts", [[{}, {}], [{"max_iters": 10}, {"max_iters": 9}], [{}, {"huber_delta": 1.0}],
                                  [{"gate_mode": 1}, {}], [{"precision": 1}, {}]])
def test_ranks_must_agree_on_solver_options(opts):
    """lh_create compares the solver options across ranks (one MAX all-reduce): ranks that would
    issue different collective counts per solve (or decide differently) are refused on every rank."""
    import lego_ba
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    rdzv = _rendezvous_file()
    procs = [ctx.Process(target=_create_main, args=(r, 2, rdzv, opts, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(2):
            r, st = q.get(timeout=100)
            got[r] = st
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        if os.path.exists(rdzv):
            os.unlink(rdzv)
    want = lego_ba.LH_OK if opts[0] == opts[1] else lego_ba.LH_E_BADARG
    assert got == {0: want, 1: want}


def test_a_failing_rank_does_not_strand_the_others():
    """lh_upload of a sharded window holds one collective (the MAX all-reduce of the envelope of S).  A
    rank whose upload fails before it (here a pixel no float holds, refused by the planner's fill) still
    joins it with its status, and every rank returns that status: no rank is left blocked in the
    collective, or in the first trial's exchange of a solve its peer never starts."""
    import lego_ba
    out = run_sharded("C2", 0, "stable_noout", corrupt_rank=1, timeout=60)
    assert out[0]["status"] == out[1]["status"] == lego_ba.LH_E_BADARG


@pytest.mark.parametrize("cfg,seed,family,th", [("C2", 1, "default", 5.991), ("mini", 2, "default", 5.991),
                                                 ("C2", 0, "stable_noout", 1e-6)])
def test_sharded_outlier_pass_equals_the_whole_window(cfg, seed, family, th):
    """Backend::Optimize's outlier pass (backend_lego.cpp:163-194) counts the whole window's edges: on a sharded
    handle each rank counts its own, the counts are summed over the ranks (one exchange of 6 doubles), and each
    rank flags its edges at the threshold the totals give.  The flags (rank 0's shard then rank 1's: the window
    order), the threshold and the counts must equal lh_classify_outliers on the two ranks' rho0 taken together,
    and every rank must report the same threshold and counts.  (th 1e-6: the doubling loop runs out.)"""
    import lego_ba
    out = run_sharded(cfg, seed, family, outlier_th=th)
    a, b = out[0], out[1]
    assert a["status"] == b["status"] == 0
    rho = np.concatenate([a["edge_robust_chi2"], b["edge_robust_chi2"]])
    flags, th_ref, n_in, n_out = lego_ba.classify_outliers(rho, th)
    assert np.array_equal(np.concatenate([a["is_outlier"], b["is_outlier"]]).astype(bool), flags)
    for r in (a, b):
        assert (r["outlier_th"], r["n_inlier"], r["n_outlier"]) == (th_ref, n_in, n_out)
    assert a["exchanges"] == b["exchanges"] == a["chains"] + 1   # the pass's exchange is not a solve collective


@pytest.mark.parametrize("case", [0, 3, 4, 8])
def test_sharded_lambda_ladder_is_bitwise_the_serial_chain(case):
    """A sharded solve's controller takes the LM decision itself (after the exchange): its workgroup 0 publishes the
    decision to the lambda ladder's rung workgroups (ladder_publish / ladder_wait).  Every rank's solve must equal
    the one-rung run (LH_NO_LADDER=1) bit for bit, the exchanges included, on windows that reject (tests/windows.py
    RELIN_WINDOWS: k_ctrl LDL^T and PCG -- decided on k_ctrl's decider workgroup --, k_ctrl_b and k_ctrl_p sharded
    two ways)."""
    from windows import RELIN_WINDOWS
    _, gen, opt, _, _ = RELIN_WINDOWS[case]
    gen = dict(gen)
    seed = gen.pop("seed")
    lad = run_sharded(gen, seed, None, max_iters=3, env={"LH_NO_BATCH": "1"}, **opt)
    one = run_sharded(gen, seed, None, max_iters=3, env={"LH_NO_LADDER": "1"}, **opt)
    for r in (0, 1):
        a, b = lad[r], one[r]
        for k in ("iterations", "trials", "accepted", "chi2_final", "lambda_final", "exchanges", "chains"):
            assert a[k] == b[k], (r, k)
        for k in ("pose_Tcw", "lm_xyz", "edge_robust_chi2", "trace_chi2"):
            assert np.array_equal(a[k], b[k]), (r, k)
    assert lad[0]["trials"] > lad[0]["accepted"]   # the windows reject (so rungs are used)
    # and batched (the default): the rungs' scalars ride behind the exchanged system and the
    # controller decides the batch after the exchange: the same solve bit for bit, in fewer chains (exchanges)
    bat = run_sharded(gen, seed, None, max_iters=3, **opt)
    for r in (0, 1):
        a, b = bat[r], one[r]
        for k in ("iterations", "trials", "accepted", "chi2_final", "lambda_final"):
            assert a[k] == b[k], (r, k)
        for k in ("pose_Tcw", "lm_xyz", "edge_robust_chi2", "trace_chi2"):
            assert np.array_equal(a[k], b[k]), (r, k)
        assert a["batch"][0] == 10 and a["batch"][1] > 0, (r, a["batch"])
        # (a batch replaces its rungs' chains by one; an acceptance at its first rung costs the same chains as the
        # serial run's evaluate-only acceptance and re-linearisation, and one stopping the loop one chain more)
        assert a["exchanges"] == a["chains"] + 1 and a["chains"] <= b["chains"] + a["batch"][1], (r, a["chains"], b["chains"])


@pytest.mark.parametrize("cfg,seed,family", [("C2", 0, "stable_noout"), ("mini", 2, "default")])
def test_p2p_exchange_matches_the_host_transport(cfg, seed, family):
    """LH_COMM_P2P: every rank writes its partial reduced system into every rank's IPC-mapped exchange buffer and
    sums the slots in rank order on the device (k_p2p_push / k_p2p_sum), the caller's all-reduce carrying only the
    bootstrap.  Two processes on the one GPU of a test box: the solve must equal the host transport's bit for bit
    (two ranks: a + b either way), with the same exchange count.  A runtime that refuses to map the other
    process's buffer on the same device makes lh_upload return LH_E_UNSUPPORTED on both ranks: recorded as a skip,
    not a pass."""
    import lego_ba
    host = run_sharded(cfg, seed, family)
    p2p = run_sharded(cfg, seed, family, comm_mode=lego_ba.LH_COMM_P2P)
    if p2p[0]["status"] == lego_ba.LH_E_UNSUPPORTED:
        assert p2p[1]["status"] == lego_ba.LH_E_UNSUPPORTED
        pytest.skip("same-device IPC mapping refused by the runtime (LH_COMM_P2P untested here)")
    for r in (0, 1):
        a, b = p2p[r], host[r]
        assert a["status"] == b["status"] == 0
        for k in ("iterations", "trials", "accepted", "chi2_initial", "chi2_final", "lambda_final", "chains"):
            assert a[k] == b[k], (r, k)
        for k in ("pose_Tcw", "lm_xyz", "edge_robust_chi2", "trace_chi2", "trace_lambda"):
            assert np.array_equal(a[k], b[k]), (r, k)
        # the host transport exchanges synchronously (one per chain); the device exchange, like RCCL, keeps two chains
        # enqueued ahead and tops every rank up to the same count after the stop
        assert b["exchanges"] == b["chains"] + 1
        assert a["exchanges"] == 1 + min(a["chains"] + 2, 10 * (10 + 1)), (a["exchanges"], a["chains"])


def test_a_rank_failing_after_the_upload_collective_takes_the_others_down():
    """A rank can fail after the envelope collective too (its controller buffers, the image initialisation, the
    copies: here lh_host.cpp's test hook), when its peers have passed it.  The upload's closing status
    all-reduce hands every rank that status, so no rank starts a solve whose exchange its peer never joins."""
    import lego_ba
    out = run_sharded("C2", 0, "stable_noout", fail_after_rank=1, timeout=60)
    assert out[0]["status"] == out[1]["status"] == lego_ba.LH_E_HIP


def _generated_one_rank(spec, seed, **opts):
    import lego_ba
    w = sharded_generated(spec, 0, spec["L"], seed)
    s = lego_ba.Solver(**opts)
    r = s.solve(w)
    r["controller"] = s.controller()
    s.close()
    return w, r


@pytest.mark.timeout(400)
@pytest.mark.parametrize("P,L,seed", [(64, 6000, 2), (128, 8000, 1)])
def test_two_rank_sharded_banded_ldlt(P, L, seed):
    """The banded LDL^T controller (k_ctrl_b, the reference's live solver problem.cpp:420) on a sharded
    window: each rank factors the all-reduced system over the union envelope of the ranks' blocks and
    takes the LM decision on the all-reduced chi2.  Gate mode 1 (the Huber gate's rounding residue
    taken as 0): the oracle's LDLT at the north-star bar and the one-rank solve to summation order."""
    import oracle_bind as ob
    spec = stable_generated(P, L)
    w, one = _generated_one_rank(spec, seed, gate_mode=1)
    assert one["controller"] == "k_ctrl_b"
    out = run_sharded(spec, seed, None, timeout=300, gate_mode=1)
    a, b = out[0], out[1]
    assert a["controller"] == b["controller"] == "k_ctrl_b"
    assert (a["iterations"], a["trials"]) == (b["iterations"], b["trials"])
    assert a["chi2_final"] == b["chi2_final"] and np.array_equal(a["pose_Tcw"], b["pose_Tcw"])
    assert a["exchanges"] == b["exchanges"] == a["chains"] + 1 and a["chains"] + 15 * a["batch"][1] >= a["trials"]
    assert (a["iterations"], a["trials"]) == (one["iterations"], one["trials"])
    assert rel(a["chi2_final"], one["chi2_final"]) < 1e-9
    assert np.allclose(a["pose_Tcw"], one["pose_Tcw"], atol=1e-9)
    o = ob.solve(w, gate_mode=1)
    assert (a["iterations"], a["trials"]) == (o["iterations"], o["trials"])
    assert rel(a["chi2_final"], o["chi2_final"]) < 1e-6
    assert np.allclose(a["pose_Tcw"], o["pose_Tcw"], atol=1e-6)
    lm = np.vstack([a["lm_xyz"], b["lm_xyz"]])
    assert np.allclose(lm, o["lm_xyz"], atol=1e-6)


@pytest.mark.timeout(400)
def test_two_rank_sharded_pcg_past_64_keyframes():
    """A sharded window past 64 keyframes on PCG (k_ctrl_p): the block list is rank-invariant (every pair
    within 64 poses, lh_plan.cpp), so both ranks all-reduce the same compact buffer.  Against the
    one-rank PCG solve and the oracle's PCG."""
    import lego_ba
    import oracle_bind as ob
    spec = stable_generated(96, 6000)
    w, one = _generated_one_rank(spec, 1, linear_solver=lego_ba.LH_SOLVER_PCG)
    assert one["controller"] == "k_ctrl_p"
    out = run_sharded(spec, 1, None, timeout=300, linear_solver=lego_ba.LH_SOLVER_PCG)
    a, b = out[0], out[1]
    assert a["controller"] == b["controller"] == "k_ctrl_p"
    assert (a["iterations"], a["trials"]) == (b["iterations"], b["trials"])
    assert a["chi2_final"] == b["chi2_final"] and np.array_equal(a["pose_Tcw"], b["pose_Tcw"])
    assert (a["iterations"], a["trials"]) == (one["iterations"], one["trials"])
    assert rel(a["chi2_final"], one["chi2_final"]) < 1e-6
    o = ob.solve(w, linear_solver=1)
    assert (a["iterations"], a["trials"]) == (o["iterations"], o["trials"])
    assert rel(a["chi2_final"], o["chi2_final"]) < 1e-6
    assert np.allclose(a["pose_Tcw"], o["pose_Tcw"], atol=1e-6)

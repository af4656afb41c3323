"""CPU tests of the window planner (lego-slam_amd/csrc/lh_plan.cpp through liblego_plan.so): the
host preprocessing lh_upload does before its copies.  The plan is the device layout every kernel
trusts (DESIGN.md "Data layout"): each observation in exactly one slot of its landmark's aligned lane
group, meta words consistent with the window, chunk windows within the MFMA envelope, and the reduce
plan covering every (chunk, pose pair) block once, in launch order.  It must not depend on the
thread count or on the order the caller lists observations in (the reference's is hash order,
problem.cpp:285)."""
import numpy as np
import pytest

import lego_ba
from windows import window

META_VALID = 1 << 23


def check_plan(w, pl, rank_invariant=False):
    O = len(w["obs_pose"])
    L = len(w["lm_xyz"])
    P = w["n_poses"]
    meta, perm = pl["meta"], pl["obs_perm"]
    valid = (meta & META_VALID) != 0
    # every observation in exactly one slot, padding slots marked invalid
    assert np.array_equal(np.sort(perm[valid]), np.arange(O))
    assert np.all(perm[~valid] == -1)
    o = perm[valid]
    m = meta[valid]
    assert np.array_equal(m & 0xFFF, w["obs_pose"][o])
    assert np.array_equal((m >> 12) & 0xF, w["obs_cam"][o])
    assert np.array_equal(pl["uv"][valid], w["obs_uv"][o])
    # landmark records: each landmark with an edge exactly once
    lp = pl["lm_perm"]
    has_edge = np.bincount(w["obs_lm"], minlength=L) > 0
    assert np.array_equal(np.sort(lp[lp >= 0]), np.flatnonzero(has_edge))
    # slot -> (sub-batch, landmark-in-sub-batch): the landmark's aligned lane group
    slots = np.flatnonzero(valid)
    sb = slots // 64
    lms = (m >> 20) & 0x7
    lg = pl["sbs"]["lg"][sb]
    assert np.all((slots % 64) >> lg == lms)
    assert np.array_equal(lp[sb * 8 + lms], w["obs_lm"][o])
    assert np.all(lms < pl["sbs"]["n_lm"][sb])
    # a landmark's observations in ascending pose order within its group
    key = sb * 8 + lms
    same = key[1:] == key[:-1]
    assert np.all(w["obs_pose"][o][1:][same] > w["obs_pose"][o][:-1][same])
    # chunks: window poses, T = ceil(6U / 16), grouped by T in launch order
    ch = pl["chunks"]
    assert np.all(ch["U"] <= 16) and np.all(ch["T"] == (6 * ch["U"].astype(int) + 15) // 16)
    assert np.all(np.diff(ch["T"].astype(int)) >= 0)
    tg = pl["tgroup_begin"]
    for T in range(1, 7):
        assert np.all(ch["T"][tg[T]:tg[T + 1]] == T)
    chunk_of_sb = np.repeat(np.arange(len(ch)), ch["sb_end"] - ch["sb_begin"])
    assert np.array_equal(ch["sb_begin"][1:], ch["sb_end"][:-1]) and ch["sb_end"][-1] == len(pl["sbs"])
    c = chunk_of_sb[sb]
    window_slot = (m >> 16) & 0xF
    assert np.array_equal(ch["pose"][c, window_slot], w["obs_pose"][o])
    # reduce plan: one pair row per (chunk, slot pair of its window); pair b owns rows
    # ptr[b] .. ptr[b+1], in launch order; items[] maps each chunk's slot pairs to their rows
    items, ptr, pq = pl["items"].astype(np.int64), pl["pair_ptr"].astype(np.int64), pl["pair_pq"]
    if P <= 64:   # the dense packed layout: every pose pair (p <= q) a block
        assert len(pq) == P * (P + 1) // 2
        bidx = lambda p, q: p * P - p * (p - 1) // 2 + (q - p)  # noqa: E731
    else:         # block-sparse: the pairs some chunk couples plus every diagonal block, sorted
        keys = [(int(a), int(b)) for a, b in pq]
        assert keys == sorted(set(keys)) and all(a <= b for a, b in keys)
        assert {(p, p) for p in range(P)} <= set(keys)
        if rank_invariant:   # every pair within the 64-pose span, whatever the shard holds
            assert keys == [(p, q) for p in range(P) for q in range(p, min(P, p + 64))]
        where = {k: i for i, k in enumerate(keys)}
        bidx = lambda p, q: where[(p, q)]  # noqa: E731
    assert ptr[-1] == len(items)
    U = ch["U"].astype(np.int64)
    expect = U * (U + 1) // 2
    assert len(items) == expect.sum()
    assert np.array_equal(ch["item_base"].astype(np.int64), np.concatenate([[0], np.cumsum(expect)[:-1]]))
    assert np.array_equal(np.sort(items), np.arange(len(items)))       # every row written once
    pair_of = np.zeros(len(items), np.int64)
    chunk_of_row = np.zeros(len(items), np.int64)
    for ci in range(len(ch)):
        k = int(ch["item_base"][ci])
        for s in range(U[ci]):
            for t in range(s, U[ci]):
                p, q = int(ch["pose"][ci, s]), int(ch["pose"][ci, t])
                b = bidx(p, q)
                r = items[k]
                assert ptr[b] <= r < ptr[b + 1] and tuple(pq[b]) == (p, q)
                chunk_of_row[r] = ci
                k += 1
    for b in range(len(pq)):
        assert np.all(np.diff(chunk_of_row[ptr[b]:ptr[b + 1]]) > 0)     # launch order within a pair
    assert np.array_equal(pl["lm_xyz"], w["lm_xyz"])


@pytest.mark.parametrize("cfg,seed,kw", [("C1", 0, {}), ("mini", 1, {}), ("C2", 2, {}),
                                         ("C2", 3, dict(pose_mode=1, k_min=2, k_max=10)),
                                         ("mini", 4, dict(pose_mode=1, k_min=1, k_max=16))])
def test_plan_invariants(cfg, seed, kw):
    w = window(cfg, seed=seed, **kw)
    pl = lego_ba.plan_window(w, threads=3)
    check_plan(w, pl)


def test_plan_independent_of_threads_and_observation_order():
    w = window("C2", seed=1, pose_mode=1, k_min=2, k_max=12)
    a = lego_ba.plan_window(w, threads=1)
    b = lego_ba.plan_window(w, threads=6)
    for k in a:
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    perm = np.random.default_rng(3).permutation(len(w["obs_pose"]))
    w2 = dict(w)
    for k in ("obs_pose", "obs_lm", "obs_cam", "obs_uv"):
        w2[k] = w[k][perm]
    c = lego_ba.plan_window(w2, threads=4)
    check_plan(w2, c)
    # identical layout; the slot -> observation map goes through the permutation
    for k in ("chunks", "sbs", "meta", "uv", "lm_perm", "items", "pair_ptr"):
        assert np.array_equal(a[k], c[k]), k
    v = a["obs_perm"] >= 0
    assert np.array_equal(perm[c["obs_perm"][v]], a["obs_perm"][v])


@pytest.mark.parametrize("chunk_lm", [8, 24, 64, 200])
def test_plan_chunk_size_option(chunk_lm):
    w = window("mini", seed=2)
    pl = lego_ba.plan_window(w, chunk_lm=chunk_lm, threads=2)
    check_plan(w, pl)
    per_chunk = [int((pl["sbs"]["n_lm"][s:e]).sum()) for s, e in zip(pl["chunks"]["sb_begin"], pl["chunks"]["sb_end"])]
    assert max(per_chunk) <= chunk_lm


def test_plan_envelope_and_errors():
    w = window("C1", seed=0)
    dup = dict(w)
    for k in ("obs_pose", "obs_lm", "obs_cam", "obs_uv"):
        dup[k] = np.concatenate([w[k], w[k][:1]])
    with pytest.raises(lego_ba.LhError) as e:
        lego_ba.plan_window(dup)
    assert e.value.status == lego_ba.LH_E_UNSUPPORTED           # two edges landmark -> same pose
    bad = dict(w, obs_lm=w["obs_lm"].copy())
    bad["obs_lm"][3] = len(w["lm_xyz"])
    with pytest.raises(lego_ba.LhError) as e:
        lego_ba.plan_window(bad)
    assert e.value.status == lego_ba.LH_E_BADARG
    empty = dict(w)
    for k in ("obs_pose", "obs_lm", "obs_cam", "obs_uv"):
        empty[k] = w[k][:0]
    with pytest.raises(lego_ba.LhError) as e:
        lego_ba.plan_window(empty)
    assert e.value.status == lego_ba.LH_E_EMPTY                 # problem.cpp:157-161
    wide = lego_ba.generate_window(P=20, L=50, k=17, seed=1, pose_mode=1)
    with pytest.raises(lego_ba.LhError) as e:
        lego_ba.plan_window(wide)
    assert e.value.status == lego_ba.LH_E_UNSUPPORTED           # > 16 poses per landmark
    for P in (64, 65, 128, 256):   # dense pair layout up to 64 poses, block-sparse past it
        wp = lego_ba.generate_window(P=P, L=40 * P, k=8, seed=1)
        check_plan(wp, lego_ba.plan_window(wp, threads=2))
    p257 = lego_ba.generate_window(P=256, L=50, k=8, seed=1)
    p257["pose_Tcw"] = np.vstack([p257["pose_Tcw"], p257["pose_Tcw"][-1:]])   # an unobserved 257th pose
    p257["n_poses"] = 257
    with pytest.raises(lego_ba.LhError) as e:
        lego_ba.plan_window(p257)
    assert e.value.status == lego_ba.LH_E_UNSUPPORTED           # > LH_PMAX_ANY poses
    span = lego_ba.generate_window(P=100, L=20, k=8, seed=1)
    span["obs_pose"] = span["obs_pose"].copy()
    first = np.flatnonzero(span["obs_lm"] == 0)
    span["obs_pose"][first[-1]] = 99                              # landmark 0 seen by poses 0.. and 99
    assert span["obs_pose"][first[0]] < 99 - 63
    with pytest.raises(lego_ba.LhError) as e:
        lego_ba.plan_window(span)
    assert e.value.status == lego_ba.LH_E_UNSUPPORTED           # a landmark spans > 64 keyframes


def test_plan_unobserved_landmarks_and_fixed_mask():
    w = window("C1", seed=1, family="stable")
    w["lm_xyz"] = np.vstack([w["lm_xyz"], [[1.0, 2.0, 3.0]], w["lm_xyz"][:2]])
    pl = lego_ba.plan_window(w)
    check_plan(w, pl)
    assert pl["fixed_mask"] == 1
    assert np.all(np.isin(np.arange(len(w["lm_xyz"]) - 3, len(w["lm_xyz"])), pl["lm_perm"], invert=True))


def test_pool_back_to_back_jobs():
    """The planner's persistent worker pool runs several jobs per upload back to back.  A worker
    that wakes after run() has retired a job must never touch it (round-2 GPU segfault: a late
    worker called through the cleared job pointer with the next job's index counter)."""
    import lego_ba
    for n in (2, 3, 17):
        runs = 20000
        assert lego_ba.pool_stress(8, runs, n) == runs * n * (n - 1) // 2


@pytest.mark.parametrize("bad", [0.1, float("nan"), 1e300, float("inf"), -float("inf"), 3.5e38])
def test_pixels_must_be_float_values(bad):
    """obs_uv is toVec2 of a cv::KeyPoint's float pixel (algorithm.h:37); the device keeps pixels as floats,
    so a measurement no float holds exactly is refused rather than silently rounded."""
    w = window("C1", seed=0)
    assert np.array_equal(w["obs_uv"].astype(np.float32).astype(np.float64), w["obs_uv"])
    lego_ba.plan_window(w)
    w["obs_uv"] = w["obs_uv"].copy()
    w["obs_uv"][17, 1] = bad
    with pytest.raises(lego_ba.LhError) as e:
        lego_ba.plan_window(w)
    assert e.value.status == lego_ba.LH_E_BADARG


def test_sharded_block_list_is_rank_invariant():
    """Past 64 poses the reduced system keeps only the blocks some chunk couples.  A
    landmark-sharded solve all-reduces that packed buffer every trial, so each rank must lay out the
    same blocks although it plans only its own landmarks: world_size > 1 handles list every pair
    within the 64-pose span (shards with different lists would sum unrelated blocks)."""
    P, L = 80, 3200
    w = lego_ba.generate_window(P=P, L=L, k=8, seed=3)
    first = np.full(L, P)
    np.minimum.at(first, w["obs_lm"], w["obs_pose"])
    shards = []
    for keep in (first < P // 2, first >= P // 2):   # shards that couple different pose pairs
        idx = np.flatnonzero(keep)
        remap = np.full(L, -1)
        remap[idx] = np.arange(len(idx))
        o = keep[w["obs_lm"]]
        s = dict(w, lm_xyz=w["lm_xyz"][idx], obs_lm=remap[w["obs_lm"][o]].astype(w["obs_lm"].dtype))
        for k in ("obs_pose", "obs_cam", "obs_uv"):
            s[k] = w[k][o]
        shards.append(s)
    own = [lego_ba.plan_window(s, threads=2) for s in shards]
    inv = [lego_ba.plan_window(s, threads=2, rank_invariant=True) for s in shards]
    for s, pl in zip(shards, inv):
        check_plan(s, pl, rank_invariant=True)
    assert np.array_equal(inv[0]["pair_pq"], inv[1]["pair_pq"])
    # the per-shard lists differ (what made the unguarded all-reduce wrong) and each is a subset
    assert not np.array_equal(own[0]["pair_pq"], own[1]["pair_pq"])
    full = {tuple(map(int, k)) for k in inv[0]["pair_pq"]}
    for pl in own:
        assert {tuple(map(int, k)) for k in pl["pair_pq"]} <= full

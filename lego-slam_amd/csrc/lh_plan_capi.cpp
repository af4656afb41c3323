// lh_plan_capi.cpp — C entry points of the window planner for the CPU test suite and the host-side
// preprocessing timings (liblego_plan.so, built with g++ only: no HIP, no GPU).  Not part of the
// solver ABI (include/lego_ba.h); the solver links lh_plan.cpp directly.
#include <chrono>
#include <cstring>
#include <vector>

#include "lh_plan.h"

namespace {
double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

extern "C" {

// sizes[0..6] = n_chunks, n_sb, n_items, npairs, n_rec, n_slots, fixed_mask; tgroup[0..LH_TMAX+1]
// rank_invariant: the block list a landmark-sharded (world_size > 1) handle uses past LH_PMAX_WIN poses
int lhp_plan_sizes(const lh_window* w, int chunk_lm, int threads, int64_t* sizes, int32_t* tgroup, int rank_invariant) {
    lh::Pool pool(threads > 0 ? threads : 1);
    lh::Plan pl;
    lh::PlanCfg cfg;
    cfg.chunk_lm = chunk_lm;
    cfg.rank_invariant_pairs = rank_invariant != 0;
    const int st = lh::plan_structure(w, cfg, false, pl, &pool);
    if (st != LH_OK) return st;
    const int64_t v[7] = {pl.n_chunks, pl.n_sb, pl.n_items, pl.npairs, pl.n_rec, pl.n_slots, (int64_t)pl.fixed_mask};
    std::memcpy(sizes, v, sizeof(v));
    for (int i = 0; i < LH_TMAX + 2; ++i) tgroup[i] = pl.tgroup_begin[i];
    return LH_OK;
}

int lhp_plan_fill(const lh_window* w, int chunk_lm, int threads, lh_chunk* chunks, lh_subbatch* sbs, uint32_t* meta,
                  float* uv, int32_t* obs_perm, int32_t* lm_perm, uint32_t* pair_ptr, uint32_t* items,
                  uint16_t* pair_pq, uint32_t* rsmap, double* lm_xyz, int rank_invariant) {
    lh::Pool pool(threads > 0 ? threads : 1);
    lh::Plan pl;
    lh::PlanCfg cfg;
    cfg.chunk_lm = chunk_lm;
    cfg.rank_invariant_pairs = rank_invariant != 0;
    const int st = lh::plan_structure(w, cfg, false, pl, &pool);
    if (st != LH_OK) return st;
    lh::PlanOut po{chunks, sbs, meta, uv, obs_perm, lm_perm, items, pair_pq, rsmap, lm_xyz};
    const int fs = lh::plan_fill(w, pl, po, &pool);
    std::memcpy(pair_ptr, pl.pair_ptr.data(), pl.pair_ptr.size() * sizeof(uint32_t));
    return fs;
}

// mean over reps plans (after one warm-up) on a persistent pool: ms of plan_structure and of
// plan_fill into reused buffers, i.e. what lh_upload spends before its copies
// diagnostic: plan_structure's stage end times (ms from its start): index checks, CSR, per-landmark
// sort + masks, span order, chunking, sub-batches, reduce-plan sizes; the last run of reps
int lhp_plan_stages(const lh_window* w, int threads, int reps, double* out7) {
    if (reps < 0 || !out7) return LH_E_BADARG;
    lh::Pool pool(threads > 0 ? threads : 1);
    lh::Plan pl;
    lh::PlanCfg cfg;
    for (int r = 0; r <= reps; ++r) {
        const int st = lh::plan_structure(w, cfg, false, pl, &pool);
        if (st != LH_OK) return st;
    }
    for (int i = 0; i < 7; ++i) out7[i] = pl.t_stage[i];
    return LH_OK;
}

int lhp_plan_time(const lh_window* w, int chunk_lm, int threads, int reps, double* ms_structure, double* ms_fill) {
    if (reps < 1 || !ms_structure || !ms_fill) return LH_E_BADARG;
    lh::Pool pool(threads > 0 ? threads : 1);
    lh::Plan pl;
    lh::PlanCfg cfg;
    cfg.chunk_lm = chunk_lm;
    std::vector<lh_chunk> chunks;
    std::vector<lh_subbatch> sbs;
    std::vector<uint32_t> meta, items, rsmap;
    std::vector<float> uv;
    std::vector<double> lm;
    std::vector<int32_t> operm, lperm;
    std::vector<uint16_t> pq;
    double ts = 0.0, tf = 0.0;
    for (int r = 0; r <= reps; ++r) {
        const double t0 = now_ms();
        const int st = lh::plan_structure(w, cfg, false, pl, &pool);
        if (st != LH_OK) return st;
        const double t1 = now_ms();
        chunks.resize(pl.n_chunks); sbs.resize(pl.n_sb); meta.resize(pl.n_slots); uv.resize(2 * pl.n_slots);
        operm.resize(pl.n_slots); lperm.resize(pl.n_rec); items.resize(pl.n_items); pq.resize(2 * (size_t)pl.npairs);
        rsmap.resize((size_t)pl.npairs * 36); lm.resize(3 * (size_t)pl.L);
        const double t2 = now_ms();
        lh::PlanOut po{chunks.data(), sbs.data(), meta.data(), uv.data(), operm.data(), lperm.data(), items.data(),
                       pq.data(), rsmap.data(), lm.data()};
        lh::plan_fill(w, pl, po, &pool);
        const double t3 = now_ms();
        if (r > 0) { ts += t1 - t0; tf += t3 - t2; }
    }
    *ms_structure = ts / reps;
    *ms_fill = tf / reps;
    return LH_OK;
}

}  // extern "C"

extern "C" {
// Pool stress for the CPU suite: `runs` back-to-back small jobs on one persistent pool (late-waking
// workers must never touch a retired job).  Returns the sum of all indices visited.
// the controllers' per-step work units (lh_common.h lh_ctrl_units) for an n-row system whose tile row I
// first reaches 8-column block fcb[I]: band 0 -> k_ctrl's table (15 unit waves, LH_NSTEP steps), band 1
// -> k_ctrl_b's (15 unit waves, the stream loaders last, 6 LH_PMAX_ANY / 8 steps).  Returns the most units a step needed.
int lhp_ctrl_units(int n, const int32_t* fcb, int band, uint16_t* units) {
    if (band) {
        const int order[LH_BAND_UNIT_WAVES] = LH_ORDER_BAND;   // as lh_host.cpp: the 11 unit waves, else the loaders too
        const int w = lh_ctrl_units(n, fcb, order, 11, 6 * LH_PMAX_ANY / 8, units);
        return w <= 11 ? w : lh_ctrl_units(n, fcb, order, LH_BAND_UNIT_WAVES, 6 * LH_PMAX_ANY / 8, units);
    }
    const int order[15] = LH_ORDER_CTRL;
    return lh_ctrl_units(n, fcb, order, 15, LH_NSTEP, units);
}

// k_ctrl's two-chain schedule (lh_ctrl_nd_plan) for tests: info = {nsteps, a, s, long_first}, units
// [16 * LH_NSTEP], pos [P]
int lhp_ctrl_nd(int P, const int32_t* pf, int32_t* info, uint16_t* units, uint8_t* pos) {
    lh_ctrl_nd nd{};
    std::vector<int> f(pf, pf + P);
    lh_ctrl_nd_plan(P, f.data(), nd);
    info[0] = nd.nsteps; info[1] = nd.a; info[2] = nd.s; info[3] = nd.long_first;
    std::memcpy(units, nd.units, sizeof(nd.units));
    for (int p = 0; p < P && p < LH_PMAX; ++p) pos[p] = nd.pos[p];
    return nd.nsteps;
}

int64_t lhp_pool_stress(int threads, int runs, int n) {
    lh::Pool pool(threads > 0 ? threads : 1);
    std::atomic<int64_t> s{0};
    for (int r = 0; r < runs; ++r) pool.run(n, [&](int i) { s += i; });
    return s.load();
}
}  // extern "C"

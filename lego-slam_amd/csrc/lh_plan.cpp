// lh_plan.cpp — window preprocessing (see lh_plan.h).  Pure C++17: no HIP, so the CPU test suite
// builds it into a host-only library (liblego_plan.so) and checks the plan's invariants.
#include "lh_plan.h"

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace lh {

// ---------------------------------------------------------------------------------------------
// Pool
// ---------------------------------------------------------------------------------------------
namespace {
// The CPUs that share the calling thread's last-level cache (sysfs cache/index3), within this
// process's affinity mask: distinct physical cores first (sysfs lists them before their SMT siblings),
// the calling thread's own CPU left out.  Empty when sysfs or the affinity mask cannot be read.
std::vector<int> llc_cpus() {
    std::vector<int> out;
    const int self = sched_getcpu();
    cpu_set_t mask;
    if (self < 0 || sched_getaffinity(0, sizeof(mask), &mask) != 0) return out;
    char path[96];
    std::snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", self);
    FILE* f = std::fopen(path, "r");
    if (!f) return out;
    char buf[512] = {0};
    const bool ok = std::fgets(buf, sizeof(buf), f) != nullptr;
    std::fclose(f);
    if (!ok) return out;
    for (char* tok = std::strtok(buf, ",\n"); tok; tok = std::strtok(nullptr, ",\n")) {
        int a = 0, b = 0;
        const int got = std::sscanf(tok, "%d-%d", &a, &b);
        if (got < 1) continue;
        if (got == 1) b = a;
        for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (c != self && CPU_ISSET(c, &mask)) out.push_back(c);
    }
    return out;
}
}  // namespace

// Workers are pinned to the CPUs sharing the caller's last-level cache (LH_HOST_PIN=0 leaves them to
// the scheduler): a GPU box exposes every host core to a process with a share of them, and a worker
// the scheduler puts on the other socket runs a pass's block at a fraction of the others' speed.
// Pools of one process never stack their workers: each worker takes the least-used CPU of the LLC's
// list (a process-wide count, released when the pool goes), so a second live handle's pool gets the
// next free cores, and rank processes of one box (LOCAL_RANK) break ties from disjoint offsets.
namespace {
std::mutex g_pin_mu;
std::vector<int> g_pin_use;   // per CPU id: workers of live pools pinned there (pools made on threads of
                              // different LLCs see different llc_cpus() lists, so counts key on the CPU)
}

Pool::Pool(int threads) {
    const char* pin_env = std::getenv("LH_HOST_PIN");
    const bool want_pin = !(pin_env && pin_env[0] == '0');
    const std::vector<int> cpus = want_pin ? llc_cpus() : std::vector<int>();
    int offset = 0;
    if (const char* lr = std::getenv("LOCAL_RANK")) offset = std::max(0, std::atoi(lr)) * std::max(threads - 1, 1);
    const int nc = (int)cpus.size();
    for (int i = 1; i < threads; ++i) {
        workers_.emplace_back([this] { loop(); });
        if (nc == 0) continue;
        int pick = -1;
        {
            std::lock_guard<std::mutex> g(g_pin_mu);
            for (int k = 0; k < nc; ++k) {
                const int c = cpus[(offset + k) % nc];
                if (c >= (int)g_pin_use.size()) g_pin_use.resize(c + 1, 0);
                if (pick < 0 || g_pin_use[c] < g_pin_use[pick]) pick = c;
            }
            ++g_pin_use[pick];
        }
        pinned_.push_back(pick);
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(pick, &one);
        pthread_setaffinity_np(workers_.back().native_handle(), sizeof(one), &one);   // best effort
    }
}

Pool::~Pool() {
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_.store(true);
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
    std::lock_guard<std::mutex> g(g_pin_mu);
    for (const int c : pinned_)
        if (c < (int)g_pin_use.size()) --g_pin_use[c];
}

// Hand-off protocol (every atomic seq_cst).  A worker counts itself in active_ *before* it loads
// job_, and run() clears job_ *before* it waits for active_ to drain.  So a worker that loaded the
// job pointer was counted before the clear, and run() does not return (the Job lives on its stack)
// until that worker has left; a worker counted after the clear loads nullptr (or a later job, which
// it may then help with: the same counting protects that one).
void Pool::loop() {
    uint64_t seen = 0;
    for (;;) {
        uint64_t g = gen_.load();
        for (unsigned spin = 0; g == seen && !stop_.load(); g = gen_.load()) {
            __builtin_ia32_pause();
            if (++spin >= kSpin) {
                std::unique_lock<std::mutex> lk(mu_);
                sleepers_.fetch_add(1);
                cv_.wait(lk, [&] { return stop_.load() || gen_.load() != seen; });
                sleepers_.fetch_sub(1);
            }
        }
        if (stop_.load()) return;
        seen = g;
        active_.fetch_add(1);
        if (Job* job = job_.load())
            for (int i = job->next.fetch_add(1); i < job->n; i = job->next.fetch_add(1)) (*job->fn)(i);
        active_.fetch_sub(1);
    }
}

void Pool::run(int n, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    if (workers_.empty() || n == 1) {
        for (int i = 0; i < n; ++i) fn(i);
        return;
    }
    Job job;
    job.fn = &fn;
    job.n = n;
    job_.store(&job);
    gen_.fetch_add(1);
    if (sleepers_.load() > 0) {   // a sleeper checks gen_ under mu_ before it waits: no lost wake-up
        std::lock_guard<std::mutex> g(mu_);
        cv_.notify_all();
    }
    for (int i = job.next.fetch_add(1); i < n; i = job.next.fetch_add(1)) fn(i);
    job_.store(nullptr);
    // bounded spin: a worker preempted while counted in active_ (oversubscribed or on the caller's
    // own core) must get the CPU back, so after a short pause loop the caller yields
    for (unsigned spin = 0; active_.load() != 0; ++spin) {
        if (spin < kSpin) __builtin_ia32_pause();
        else std::this_thread::yield();
    }
}

namespace {

// run fn(begin, end) over [0, n) in about 4 blocks per thread
void parallel_range(Pool* pool, int64_t n, int64_t min_block, const std::function<void(int64_t, int64_t)>& fn) {
    if (n <= 0) return;
    const int threads = pool ? pool->size() : 1;
    int64_t nb = std::max<int64_t>(1, std::min<int64_t>(4 * threads, (n + min_block - 1) / min_block));
    const int64_t bs = (n + nb - 1) / nb;
    nb = (n + bs - 1) / bs;
    auto body = [&](int b) { fn((int64_t)b * bs, std::min<int64_t>(n, (int64_t)(b + 1) * bs)); };
    if (pool) pool->run((int)nb, body);
    else for (int b = 0; b < nb; ++b) body(b);
}

inline int popc(uint64_t m) { return __builtin_popcountll(m); }
inline int chunk_tiles(uint64_t mask) { return (6 * popc(mask) + 15) / 16; }
inline int pow2log(int k) { int g = 1, lg = 0; while (g < k) { g <<= 1; ++lg; } return lg; }

// block index of pose pair (p, q), p <= q: the dense packed order up to LH_PMAX_WIN poses, else the
// position in the sorted pair list (binary search)
inline int pair_index(const Plan& pl, int p, int q) {
    if (pl.P <= LH_PMAX_WIN) return p * pl.P - (p * (p - 1)) / 2 + (q - p);
    const uint32_t key = (uint32_t)p << 16 | (uint32_t)q;
    int lo = 0, hi = pl.npairs;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        const uint32_t k = (uint32_t)pl.pair_list[2 * mid] << 16 | pl.pair_list[2 * mid + 1];
        if (k <= key) lo = mid; else hi = mid;
    }
    return lo;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// plan_structure
// ---------------------------------------------------------------------------------------------
int plan_structure(const lh_window* w, const PlanCfg& cfg, bool allow_empty, Plan& pl, Pool* pool) {
    if (!w) return LH_E_BADARG;
    if (w->n_poses < 0 || w->n_landmarks < 0 || w->n_obs < 0) return LH_E_BADARG;
    if (w->n_poses > 0 && !w->pose_Tcw) return LH_E_BADARG;
    if (w->n_landmarks > 0 && !w->lm_xyz) return LH_E_BADARG;
    if (w->n_obs > 0 && (!w->obs_pose || !w->obs_lm || !w->obs_uv)) return LH_E_BADARG;
    if (w->n_cams < 0 || (w->n_cams > 0 && !w->cam_ext)) return LH_E_BADARG;
    if (w->n_cams > LH_MAX_CAMS) return LH_E_UNSUPPORTED;   // per-(pose, camera) tables sized for 4 cameras
    const int P = w->n_poses, L = w->n_landmarks;
    const int64_t O = w->n_obs;
    const int ncam = w->n_cams > 0 ? w->n_cams : 1;
    pl.P = P; pl.L = L; pl.O = O; pl.ncam = ncam;
    const auto t_0 = std::chrono::steady_clock::now();
    auto stage = [&](int i) {
        pl.t_stage[i] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_0).count();
    };

    // ---- index checks and the landmark-major CSR, one parallel pass.  The CSR assumes the input is
    //      already grouped by landmark (what Backend::Optimize's landmark loop produces) and is rebuilt
    //      by a counting sort when it is not. ----
    std::atomic<int> bad{0}, unsorted{0};
    pl.lm_ptr.assign((size_t)L + 1, 0);
    pl.csr.resize((size_t)O);
    parallel_range(pool, O, 1 << 15, [&](int64_t b, int64_t e) {
        uint32_t prev = b > 0 ? w->obs_lm[b - 1] : 0;
        bool bd = false, us = false;
        for (int64_t o = b; o < e; ++o) {
            const uint32_t l = w->obs_lm[o];
            const bool ok = w->obs_pose[o] < (uint32_t)P && l < (uint32_t)L && (!w->obs_cam || w->obs_cam[o] < ncam);
            bd |= !ok;
            us |= l < prev;
            pl.csr[o] = o;
            // the landmarks from the previous observation's (exclusive) to this one start here.  Blocks write
            // disjoint ranges when the input is grouped by landmark; when it is not, two locally sorted blocks
            // can write one entry (ThreadSanitizer found it, scripts/sanitize.sh) before the counting sort below
            // rebuilds lm_ptr, so the stores are relaxed atomics (plain stores on x86): no data race, same code
            if (ok && !us)
                for (int64_t q = o > 0 ? (int64_t)prev + 1 : 0; q <= (int64_t)l; ++q)
                    __atomic_store_n(&pl.lm_ptr[q], (int64_t)o, __ATOMIC_RELAXED);
            prev = l;
        }
        // the measurement is a cv::KeyPoint's float pixel widened (toVec2, algorithm.h:37): the device
        // keeps it as a float, so a value a float cannot hold exactly (or a NaN) is a bad argument
        // (a loop of its own: it vectorises).  Only in-range finite values are converted: the
        // double -> float conversion of a value past FLT_MAX is undefined, and +-inf would compare equal.
        for (int64_t i = 2 * b; i < 2 * e; ++i) {
            const double x = w->obs_uv[i];
            const bool fin = std::fabs(x) <= (double)FLT_MAX;
            bd |= !(fin && (double)(float)(fin ? x : 0.0) == x);
        }
        if (bd) bad.store(1);
        if (us) unsorted.store(1);
    });
    if (bad.load()) return LH_E_BADARG;
    if (!allow_empty && (O == 0 || (P + L) == 0)) return LH_E_EMPTY;   // problem.cpp:157-161
    if (P > LH_PMAX_ANY) return LH_E_UNSUPPORTED;   // the reduced solve's LDS vectors (k_ctrl_p)
    if (O >= (int64_t)1 << 30) return LH_E_UNSUPPORTED;                 // int32 slot indices
    pl.fixed_bits.assign((size_t)(P + 63) / 64 + 1, 0ull);
    if (w->pose_fixed)
        for (int p = 0; p < P; ++p)
            if (w->pose_fixed[p]) pl.fixed_bits[p >> 6] |= 1ull << (p & 63);
    pl.fixed_mask = pl.fixed_bits[0];

    stage(0);
    if (!unsorted.load()) {
        for (int64_t l = (O > 0 ? (int64_t)w->obs_lm[O - 1] + 1 : 0); l <= L; ++l) pl.lm_ptr[l] = O;
    } else {
        std::fill(pl.lm_ptr.begin(), pl.lm_ptr.end(), 0);
        for (int64_t o = 0; o < O; ++o) pl.lm_ptr[w->obs_lm[o] + 1]++;
        for (int l = 0; l < L; ++l) pl.lm_ptr[l + 1] += pl.lm_ptr[l];
        std::vector<int64_t> pos(pl.lm_ptr.begin(), pl.lm_ptr.end() - 1);
        for (int64_t o = 0; o < O; ++o) pl.csr[pos[w->obs_lm[o]]++] = o;
    }

    stage(1);
    // ---- per landmark: ascending pose order, pose mask, envelope checks ----
    pl.lm_mask.assign((size_t)L, 0ull);
    pl.lm_base.assign((size_t)L, 0);
    std::atomic<int> unsup{0};
    parallel_range(pool, L, 4096, [&](int64_t b, int64_t e) {
        bool us = false;
        for (int64_t l = b; l < e; ++l) {
            int64_t* s = pl.csr.data() + pl.lm_ptr[l];
            const int64_t k = pl.lm_ptr[l + 1] - pl.lm_ptr[l];
            if (k > LH_SB_OBS) { us = true; continue; }
            for (int64_t i = 1; i < k; ++i) {   // insertion sort by (pose, window index)
                const int64_t v = s[i];
                const uint32_t pv = w->obs_pose[v];
                int64_t j = i - 1;
                while (j >= 0 && (w->obs_pose[s[j]] > pv || (w->obs_pose[s[j]] == pv && s[j] > v))) { s[j + 1] = s[j]; --j; }
                s[j + 1] = v;
            }
            // observing poses relative to the first one (ascending): bit i = pose base + i; a landmark
            // must be seen within 64 consecutive keyframes (a sliding window's are, map.h:82)
            uint64_t m = 0;
            const int base = k > 0 ? (int)w->obs_pose[s[0]] : 0;
            for (int64_t i = 0; i < k; ++i) {
                const uint32_t rel = w->obs_pose[s[i]] - (uint32_t)base;
                if (rel >= 64) { us = true; break; }
                const uint64_t bit = 1ull << rel;
                if (m & bit) us = true;   // two edges landmark -> same pose (DESIGN.md "Limits")
                m |= bit;
            }
            if (popc(m) > LH_UMAX) us = true;
            pl.lm_mask[l] = m;
            pl.lm_base[l] = base;
        }
        if (us) unsup.store(1);
    });
    if (unsup.load()) return LH_E_UNSUPPORTED;

    stage(2);
    std::vector<uint64_t>& om = pl.ord_mask;
    std::vector<int32_t>& ob = pl.ord_base;
    std::vector<uint8_t>& olg = pl.ord_lg;
    // ---- landmark order by observation span (first pose, last pose, mask), stable: a parallel
    //      counting sort (per-block histograms, prefix in bucket-major / block-minor order, so each
    //      bucket keeps landmark order), then a stable sort by mask inside the buckets that mix masks ----
    {
        // bucket (first pose, span): the order of (first pose, last pose), with P x 64 buckets
        const int nb = std::max(P, 1) * 64;
        auto bucket = [&](int l) {
            const uint64_t m = pl.lm_mask[l];   // bit 0 is the first pose
            return pl.lm_base[l] * 64 + (63 - __builtin_clzll(m));
        };
        const int threads = pool ? pool->size() : 1;
        const int nblk = std::max(1, std::min(4 * threads, (L + 8191) / 8192));
        const int bsz = (L + nblk - 1) / std::max(nblk, 1);
        std::vector<int32_t> hist((size_t)nblk * (nb + 1), 0);
        auto count_blk = [&](int k) {
            int32_t* h = hist.data() + (size_t)k * (nb + 1);
            const int l0 = k * bsz, l1 = std::min(L, l0 + bsz);
            for (int l = l0; l < l1; ++l)
                if (pl.lm_mask[l]) h[bucket(l)]++;   // edge-less landmarks are no vertex (backend_lego.cpp:126)
        };
        if (pool) pool->run(nblk, count_blk);
        else for (int k = 0; k < nblk; ++k) count_blk(k);
        int32_t run = 0;
        for (int bk = 0; bk < nb; ++bk)
            for (int k = 0; k < nblk; ++k) {
                int32_t& h = hist[(size_t)k * (nb + 1) + bk];
                const int32_t c = h;
                h = run;
                run += c;
            }
        const int Lact0 = run;
        pl.order.resize((size_t)Lact0);
        om.resize((size_t)Lact0);
        ob.resize((size_t)Lact0);
        olg.resize((size_t)Lact0);
        // the chunking pass reads each landmark's mask, first pose and lane-group log in span order:
        // written here with the order itself
        auto put = [&](int32_t i, int l) {
            pl.order[i] = l;
            om[i] = pl.lm_mask[l];
            ob[i] = pl.lm_base[l];
            olg[i] = (uint8_t)pow2log((int)(pl.lm_ptr[l + 1] - pl.lm_ptr[l]));
        };
        auto scatter_blk = [&](int k) {
            int32_t* h = hist.data() + (size_t)k * (nb + 1);
            const int l0 = k * bsz, l1 = std::min(L, l0 + bsz);
            for (int l = l0; l < l1; ++l)
                if (pl.lm_mask[l]) put(h[bucket(l)]++, l);
        };
        if (pool) pool->run(nblk, scatter_blk);
        else for (int k = 0; k < nblk; ++k) scatter_blk(k);
        // bucket bounds: after the scatter, block nblk-1's cursor of bucket bk is the bucket's end
        std::vector<int32_t> bend((size_t)nb);
        for (int bk = 0; bk < nb; ++bk) bend[bk] = hist[(size_t)(nblk - 1) * (nb + 1) + bk];
        auto sort_bucket = [&](int bk) {
            const int32_t e0 = bend[bk], s0 = bk > 0 ? bend[bk - 1] : 0;
            auto s = pl.order.begin() + s0, e = pl.order.begin() + e0;
            if (e - s < 2) return;
            const uint64_t m0 = pl.lm_mask[*s];
            if (std::all_of(s, e, [&](int32_t l) { return pl.lm_mask[l] == m0; })) return;
            std::stable_sort(s, e, [&](int32_t x, int32_t y) { return pl.lm_mask[x] < pl.lm_mask[y]; });
            for (int32_t i = s0; i < e0; ++i) put(i, pl.order[i]);
        };
        if (pool) pool->run(nb, sort_bucket);
        else for (int bk = 0; bk < nb; ++bk) sort_bucket(bk);
    }
    const int Lact = (int)pl.order.size();
    stage(3);

    // ---- chunks: at most ~512 (2 workgroups per CU, all resident at once), whole sub-batches of 8
    //      landmarks.  Rounding up to 8 rather than to 4 x 8 (equal sub-batches per wave) keeps the
    //      count near 512 (C3: 104 landmarks, 488 chunks of 13 sub-batches, so one wave in four runs
    //      a fourth sub-batch).  Rounding to 32 gives 128 (398 chunks: 142 CUs run two chunks of
    //      4 sub-batches per wave, 114 run one), and 96 gives 528 chunks (16 wait for a free slot).
    //      Measured on C3: k_lin 41.2 us at 104, 44.0 at 128, 51.6 at 96. ----
    int chunk_lm = (Lact + 511) / 512;
    chunk_lm = ((chunk_lm + LH_SB_LM - 1) / LH_SB_LM) * LH_SB_LM;
    chunk_lm = std::max(32, std::min(256, chunk_lm));
    if (cfg.chunk_lm > 0) chunk_lm = std::max(LH_SB_LM, std::min(512, cfg.chunk_lm));
    // One serial pass over the span order cuts the chunks and packs their sub-batches (the masks, first
    // poses and lane-group logs in span order, om / ob / olg, so the pass reads them sequentially).
    // A chunk's MFMA tile count T is set by the union of its landmarks' poses: start a new chunk
    // rather than let the union grow past the larger of the two tile counts.  A sub-batch takes
    // landmarks while it holds < 8 and (n + 1) << lg <= 64 (landmark l owns the aligned lane group
    // [l*G, l*G + k_l) of its 64 slots, G = 2^lg the largest pow2ceil(k) in the sub-batch).
    // The pass runs over segments of the span order in parallel, each cut where the first pose changes
    // and started as a fresh chunk; the segments are then joined only if the serial pass would have started
    // a fresh chunk at every cut too (a sliding window's chunks end where the first pose moves: the union
    // with the next run of poses raises the tile count), else the serial pass runs: the same plan either way.
    struct Cut {
        std::vector<int32_t> lm0, base, sb0, tfirst;   // sb0: relative to this segment's sub-batches
        std::vector<uint64_t> mask;
        std::vector<uint8_t> tlg;
        uint64_t cmask = 0;
        int cbase = 0, clm0 = 0, ctiles = 0;
        bool have = false;
    };
    auto fresh_at = [&](const Cut& c, int i, uint64_t& m) {
        const uint64_t oi = om[i];
        const int sh = c.have ? ob[i] - c.cbase : 64;
        m = (sh < 64 && (oi >> (63 - sh)) <= 1) ? oi << sh : 0ull;
        bool fresh = m == 0 || (i - c.clm0) >= chunk_lm;
        if (!fresh && (c.cmask | m) != c.cmask) {
            const uint64_t u = c.cmask | m;
            fresh = popc(u) > LH_UMAX || chunk_tiles(u) > std::max(c.ctiles, chunk_tiles(m));
        }
        return fresh;
    };
    auto cut_range = [&](int i0, int i1, Cut& c) {
        c.tfirst.reserve((size_t)(i1 - i0) / 4 + 8);
        c.tlg.reserve((size_t)(i1 - i0) / 4 + 8);
        int sb_start = 0, sb_n = 0, sb_lg = 0;
        auto close_sb = [&]() {
            if (sb_n > 0) { c.tfirst.push_back(sb_start); c.tlg.push_back((uint8_t)sb_lg); }
            sb_n = 0;
        };
        // the current chunk lives in c's locals and is pushed when the next one starts
        auto push_chunk = [&]() {
            if (!c.have) return;
            c.lm0.push_back(c.clm0);
            c.mask.push_back(c.cmask);
            c.base.push_back(c.cbase);
        };
        for (int i = i0; i < i1; ++i) {
            // the landmark's mask relative to the current chunk's base (landmarks come in ascending first
            // pose, so the base is the chunk's first pose); past 64 poses from the base it starts a chunk
            uint64_t m;
            if (fresh_at(c, i, m)) {
                close_sb();
                push_chunk();
                c.have = true;
                c.clm0 = i;
                c.cmask = om[i];
                c.cbase = ob[i];
                c.sb0.push_back((int32_t)c.tfirst.size());
            } else {
                c.cmask |= m;
            }
            c.ctiles = chunk_tiles(c.cmask);
            const int lgn = std::max(sb_lg, (int)olg[i]);
            if (sb_n > 0 && sb_n < LH_SB_LM && ((sb_n + 1) << lgn) <= LH_SB_OBS) {
                ++sb_n;
                sb_lg = lgn;
            } else {
                close_sb();
                sb_start = i;
                sb_n = 1;
                sb_lg = olg[i];
            }
        }
        push_chunk();
        close_sb();
    };
    // segment starts: about two per pool thread, each moved forward to the next change of first pose
    std::vector<int> seg{0};
    {
        const int want = pool ? 2 * pool->size() : 1;
        for (int k = 1; k < want; ++k) {
            int i = (int)((int64_t)Lact * k / want);
            i = std::max(i, seg.back() + 1);
            while (i < Lact && ob[i] == ob[i - 1]) ++i;
            if (i < Lact && i > seg.back()) seg.push_back(i);
        }
        seg.push_back(Lact);
    }
    const int nseg = (int)seg.size() - 1;
    std::vector<Cut> cuts((size_t)std::max(nseg, 1));
    if (pool && nseg > 1) pool->run(nseg, [&](int k) { cut_range(seg[k], seg[k + 1], cuts[k]); });
    else for (int k = 0; k < nseg; ++k) cut_range(seg[k], seg[k + 1], cuts[k]);
    bool joined = true;
    for (int k = 1; k < nseg && joined; ++k) {
        uint64_t m;
        joined = fresh_at(cuts[k - 1], seg[k], m);
    }
    if (!joined) {   // a chunk would run across a cut: the serial pass
        cuts.assign(1, Cut{});
        cut_range(0, Lact, cuts[0]);
    }
    std::vector<int32_t> c_sb0;              // per chunk (creation order): its first sub-batch
    std::vector<int32_t> t_first;            // sub-batches in creation order: first position
    std::vector<uint8_t> t_lg;
    pl.chunk_lm0.clear();
    pl.chunk_mask.clear();
    pl.chunk_base.clear();
    for (const Cut& c : cuts) {
        const int32_t off = (int32_t)t_first.size();
        for (int32_t v : c.sb0) c_sb0.push_back(v + off);
        pl.chunk_lm0.insert(pl.chunk_lm0.end(), c.lm0.begin(), c.lm0.end());
        pl.chunk_mask.insert(pl.chunk_mask.end(), c.mask.begin(), c.mask.end());
        pl.chunk_base.insert(pl.chunk_base.end(), c.base.begin(), c.base.end());
        t_first.insert(t_first.end(), c.tfirst.begin(), c.tfirst.end());
        t_lg.insert(t_lg.end(), c.tlg.begin(), c.tlg.end());
    }
    const int NC = (int)pl.chunk_mask.size();
    pl.chunk_lm0.push_back(Lact);
    c_sb0.push_back((int32_t)t_first.size());
    pl.n_chunks = NC;

    // launch order: grouped by T (one k_lin launch per tile count), stable
    pl.corder.resize((size_t)NC);
    {
        int c = 0;
        for (int T = 1; T <= LH_TMAX; ++T) {
            pl.tgroup_begin[T] = c;
            for (int i = 0; i < NC; ++i)
                if (chunk_tiles(pl.chunk_mask[i]) == T) pl.corder[c++] = i;
        }
        pl.tgroup_begin[0] = 0;
        pl.tgroup_begin[LH_TMAX + 1] = c;
    }
    stage(4);

    // ---- sub-batches in launch order ----
    pl.chunk_sb0.assign((size_t)NC + 1, 0);
    for (int ci = 0; ci < NC; ++ci) {
        const int c = pl.corder[ci];
        pl.chunk_sb0[ci + 1] = pl.chunk_sb0[ci] + (c_sb0[c + 1] - c_sb0[c]);   // by launch position
    }
    pl.n_sb = pl.chunk_sb0[NC];
    pl.n_rec = pl.n_sb * LH_SB_LM;
    pl.n_slots = (int64_t)pl.n_sb * LH_SB_OBS;
    pl.sb_lm0.resize((size_t)pl.n_sb + 1);
    pl.sb_lg.resize((size_t)pl.n_sb);
    for (int ci = 0; ci < NC; ++ci) {
        const int c = pl.corder[ci], n = c_sb0[c + 1] - c_sb0[c];
        std::memcpy(pl.sb_lm0.data() + pl.chunk_sb0[ci], t_first.data() + c_sb0[c], (size_t)n * sizeof(int32_t));
        std::memcpy(pl.sb_lg.data() + pl.chunk_sb0[ci], t_lg.data() + c_sb0[c], (size_t)n);
    }
    pl.sb_lm0[pl.n_sb] = Lact;   // never read as a start: the last sub-batch ends at its chunk's end

    stage(5);
    // ---- reduce plan sizes: the reduced system's blocks (pose pairs p <= q) and, per block, the
    //      chunks touching it.  Up to LH_PMAX_WIN poses every pair has a block (the dense packed layout
    //      k_ctrl / k_ctrl_g scatter from); past it only the pairs some chunk touches, plus every
    //      diagonal block (S is then block-sparse: a landmark couples poses within its 64-pose span) ----
    pl.pair_list.clear();
    if (P <= LH_PMAX_WIN) {
        for (int p = 0; p < P; ++p)
            for (int q = p; q < P; ++q) { pl.pair_list.push_back((uint16_t)p); pl.pair_list.push_back((uint16_t)q); }
    } else if (cfg.rank_invariant_pairs) {
        // landmark-sharded solve: every rank must lay out (and all-reduce) the same blocks, and a
        // rank sees only its own chunks, so the list is every pair a landmark could couple (a
        // landmark's poses lie within 64 consecutive keyframes), whatever this rank's shard holds
        for (int p = 0; p < P; ++p)
            for (int q = p; q < P && q - p < 64; ++q) {
                pl.pair_list.push_back((uint16_t)p);
                pl.pair_list.push_back((uint16_t)q);
            }
    } else {
        std::vector<uint32_t> keys;
        for (int p = 0; p < P; ++p) keys.push_back((uint32_t)p << 16 | (uint32_t)p);
        for (int ci = 0; ci < NC; ++ci) {
            const int c = pl.corder[ci], base = pl.chunk_base[c];
            for (uint64_t a = pl.chunk_mask[c]; a; a &= a - 1)
                for (uint64_t b = a; b; b &= b - 1)
                    keys.push_back((uint32_t)(base + __builtin_ctzll(a)) << 16 | (uint32_t)(base + __builtin_ctzll(b)));
        }
        std::sort(keys.begin(), keys.end());
        keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
        for (uint32_t k : keys) { pl.pair_list.push_back((uint16_t)(k >> 16)); pl.pair_list.push_back((uint16_t)(k & 0xFFFF)); }
    }
    pl.npairs = (int)(pl.pair_list.size() / 2);
    // block rows: pairs (p', r), p' < r, read transposed (ascending p'), then pairs (r, q'), q' >= r
    pl.brow_ptr.assign((size_t)P + 1, 0);
    for (int b = 0; b < pl.npairs; ++b) {
        const int p = pl.pair_list[2 * b], q = pl.pair_list[2 * b + 1];
        pl.brow_ptr[p + 1]++;
        if (q != p) pl.brow_ptr[q + 1]++;
    }
    for (int p = 0; p < P; ++p) pl.brow_ptr[p + 1] += pl.brow_ptr[p];
    pl.brow_ent.assign((size_t)pl.brow_ptr[P], 0u);
    {
        std::vector<int32_t> fill(pl.brow_ptr.begin(), pl.brow_ptr.end() - 1);
        for (int b = 0; b < pl.npairs; ++b) {   // transposed entries first: every pair (p', r) precedes (r, .)
            const int p = pl.pair_list[2 * b], q = pl.pair_list[2 * b + 1];
            if (q != p) pl.brow_ent[fill[q]++] = (uint32_t)b << 13 | (uint32_t)p << 1 | 1u;
        }
        for (int b = 0; b < pl.npairs; ++b) {
            const int p = pl.pair_list[2 * b], q = pl.pair_list[2 * b + 1];
            pl.brow_ent[fill[p]++] = (uint32_t)b << 13 | (uint32_t)q << 1;
        }
    }
    pl.pair_ptr.assign((size_t)pl.npairs + 1, 0u);
    for (int ci = 0; ci < NC; ++ci) {
        const int c = pl.corder[ci], base = pl.chunk_base[c];
        for (uint64_t a = pl.chunk_mask[c]; a; a &= a - 1) {
            const int p = base + __builtin_ctzll(a);
            for (uint64_t b = a; b; b &= b - 1) pl.pair_ptr[pair_index(pl, p, base + __builtin_ctzll(b)) + 1]++;
        }
    }
    for (int b = 0; b < pl.npairs; ++b) pl.pair_ptr[b + 1] += pl.pair_ptr[b];
    pl.n_items = (int)pl.pair_ptr[pl.npairs];
    pl.chunk_ib.assign((size_t)NC + 1, 0u);
    for (int ci = 0; ci < NC; ++ci) {
        const uint32_t u = (uint32_t)popc(pl.chunk_mask[pl.corder[ci]]);
        pl.chunk_ib[ci + 1] = pl.chunk_ib[ci] + u * (u + 1) / 2;
    }
    stage(6);
    return LH_OK;
}

// ---------------------------------------------------------------------------------------------
// plan_fill
// ---------------------------------------------------------------------------------------------
int plan_fill(const lh_window* w, const Plan& pl, const PlanOut& out, Pool* pool, SlotsReady on_slots, void* user,
              int batches) {
    const int P = pl.P, NC = pl.n_chunks;
    // chunks and their sub-batches' observation slots, one task per chunk
    auto chunk_task = [&](int ci) {
        const int c = pl.corder[ci];
        const uint64_t m = pl.chunk_mask[c];
        lh_chunk ck;
        std::memset(&ck, 0, sizeof(ck));
        ck.U = (uint8_t)popc(m);
        ck.T = (uint8_t)chunk_tiles(m);
        const int pbase = pl.chunk_base[c];
        int slot_of[64] = {0};   // by pose - pbase
        {
            int s = 0;
            for (uint64_t a = m; a; a &= a - 1) {
                const int r = __builtin_ctzll(a);
                ck.pose[s] = (uint16_t)(pbase + r);
                slot_of[r] = s++;
            }
        }
        ck.sb_begin = (uint32_t)pl.chunk_sb0[ci];
        ck.sb_end = (uint32_t)pl.chunk_sb0[ci + 1];
        ck.item_base = pl.chunk_ib[ci];
        out.chunks[ci] = ck;
        const int lm_end = pl.chunk_lm0[c + 1];
        for (int sb = pl.chunk_sb0[ci]; sb < pl.chunk_sb0[ci + 1]; ++sb) {
            const int first = pl.sb_lm0[sb];
            const int last = (sb + 1 < pl.chunk_sb0[ci + 1]) ? pl.sb_lm0[sb + 1] : lm_end;
            const int n = last - first, lg = pl.sb_lg[sb];
            lh_subbatch sbd;
            std::memset(&sbd, 0, sizeof(sbd));
            sbd.lm_begin = (uint32_t)sb * LH_SB_LM;
            sbd.n_lm = (uint8_t)n;
            sbd.lg = (uint8_t)lg;
            out.sbs[sb] = sbd;
            const int64_t base = (int64_t)sb * LH_SB_OBS;
            auto pad = [&](int64_t s0, int64_t s1) {   // unused slots: a meta word without LH_META_VALID
                for (int64_t s = s0; s < s1; ++s) {
                    out.meta[s] = 0u;
                    out.uv[2 * s] = 0.0f;
                    out.uv[2 * s + 1] = 0.0f;
                    out.obs_perm[s] = -1;
                }
            };
            for (int q = 0; q < LH_SB_LM; ++q) out.lm_perm[sbd.lm_begin + q] = q < n ? pl.order[first + q] : -1;
            for (int q = 0; q < n; ++q) {   // every slot is written once
                const int l = pl.order[first + q];
                int64_t slot = base + ((int64_t)q << lg);
                for (int64_t r = pl.lm_ptr[l]; r < pl.lm_ptr[l + 1]; ++r, ++slot) {
                    const int64_t o = pl.csr[r];
                    const uint32_t p = w->obs_pose[o];
                    const uint32_t cam = w->obs_cam ? w->obs_cam[o] : 0;
                    out.meta[slot] = LH_META(p, cam, slot_of[p - (uint32_t)pbase], q);
                    out.uv[2 * slot] = (float)w->obs_uv[2 * o];   // exact: checked in plan_structure
                    out.uv[2 * slot + 1] = (float)w->obs_uv[2 * o + 1];
                    out.obs_perm[slot] = (int32_t)o;
                }
                pad(slot, base + ((int64_t)(q + 1) << lg));
            }
            pad(base + ((int64_t)n << lg), base + LH_SB_OBS);
        }
    };
    // chunks in launch order own contiguous sub-batches, hence contiguous slots: batch b of the chunk
    // pass finishes slots [64 chunk_sb0[c0], 64 chunk_sb0[c1])
    const int nbat = std::max(1, std::min(batches, NC));
    for (int b = 0; b < nbat; ++b) {
        const int c0 = (int)((int64_t)NC * b / nbat), c1 = (int)((int64_t)NC * (b + 1) / nbat);
        if (pool) pool->run(c1 - c0, [&](int i) { chunk_task(c0 + i); });
        else for (int ci = c0; ci < c1; ++ci) chunk_task(ci);
        if (on_slots && c1 > c0)
            on_slots(user, (int64_t)pl.chunk_sb0[c0] * LH_SB_OBS, (int64_t)pl.chunk_sb0[c1] * LH_SB_OBS);
    }

    // reduce plan: pose pair b owns the pair rows pair_ptr[b] .. pair_ptr[b+1], one per chunk whose
    // window holds both poses, in launch order (k_reduce sums them in this order: a fixed,
    // thread-count-independent order).  items[] maps each chunk's slot pairs (s <= t, row-major
    // over its U slots, from chunk_ib) to the row k_lin writes that pair's block into.
    {
        std::vector<uint32_t> cur(pl.pair_ptr.begin(), pl.pair_ptr.end() - 1);
        for (int ci = 0; ci < NC; ++ci) {
            const int c = pl.corder[ci], base = pl.chunk_base[c];
            int ps[64], U = 0;
            for (uint64_t a = pl.chunk_mask[c]; a; a &= a - 1) ps[U++] = base + __builtin_ctzll(a);
            uint32_t k = pl.chunk_ib[ci];
            for (int s = 0; s < U; ++s)
                for (int t = s; t < U; ++t) out.items[k++] = cur[pair_index(pl, ps[s], ps[t])]++;
        }
    }
    std::memcpy(out.pair_pq, pl.pair_list.data(), pl.pair_list.size() * sizeof(uint16_t));
    // reduced-system element map for k_ctrl's register scatter: S element of pose pair (pi, pj),
    // pi <= pj, row a, col b -> global rows 6 pi + a, 6 pj + b (9 bits each), diagonal-block flag
    // (only the dense layouts, P <= LH_PMAX_WIN, are scattered; 9 bits hold rows < 512)
    if (P <= LH_PMAX_WIN)
        for (int blk = 0; blk < pl.npairs; ++blk) {
            const int pi = pl.pair_list[2 * blk], pj = pl.pair_list[2 * blk + 1];
            for (int a = 0; a < 6; ++a)
                for (int b = 0; b < 6; ++b)
                    out.rsmap[(size_t)blk * 36 + 6 * a + b] = LH_RSMAP(6 * pi + a, 6 * pj + b, pi == pj);
        }
    if (out.lm_xyz)
        parallel_range(pool, 3 * (int64_t)pl.L, 1 << 16, [&](int64_t b, int64_t e) {
            if (e > b) std::memcpy(out.lm_xyz + b, w->lm_xyz + b, (size_t)(e - b) * sizeof(double));
        });
    return LH_OK;
}

}  // namespace lh

// lh_host.cpp — C ABI (include/lego_ba.h) of the MI355X BA solver: window
// preprocessing, device buffers, the LM launch loop and the RCCL exchange.
//
// Host-side work per window (once, at lh_upload):
//   * landmark-major CSR of the observations, each landmark's observations in
//     ascending pose order (the reference visits edges in hash order; any order
//     is the same problem);
//   * landmarks sorted by observation span and packed into chunks whose union
//     of observing poses fits one MFMA window (<= LH_UMAX poses), chunks split
//     into wave sub-batches (<= 8 landmarks, <= 64 observations);
//   * the reduce plan: for every pose pair, the chunks that touch it.
// Per solve nothing but kernel launches (and, with >1 rank, one RCCL all-reduce
// per LM trial) happens on the host; it polls the device stop flag every few
// trials.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <numeric>
#include <vector>

#include "../../include/lego_ba.h"
#include "lh_common.h"

extern "C" {
hipError_t lh_prepare_lin();
size_t lh_lin_smem(int T, int ncam);
hipError_t lh_launch_nop(hipStream_t st);
hipError_t lh_launch_lin(int T, int trial, int nchunks, int chunk_base, hipStream_t st, const lh_chunk* chunks,
                         const lh_subbatch* sbs, const double* obs_uv, const uint32_t* obs_meta, double* rec,
                         const double* ptab, const double* ext, const lh_ctrl* ctrl, const double* dxp,
                         double* edge_rho, double* slabs, lh_params prm, int nrec, uint32_t fixed_mask);
hipError_t lh_launch_reduce(hipStream_t st, const lh_chunk* chunks, const double* slabs, const uint32_t* pair_ptr,
                            const uint32_t* items, const uint16_t* pair_pq, const lh_ctrl* ctrl, double* rs_stage,
                            double* maxd, lh_params prm, int n_chunks);
hipError_t lh_launch_ctrl(hipStream_t st, lh_ctrl* ctrl, double* rs_commit, const double* rs_stage, const double* maxd,
                          const uint32_t* rsmap, double* pose_qt, double* ptab, const double* ext, double* dxp,
                          lh_params prm, int mode, int* host_done, int seq);
hipError_t lh_launch_reset(hipStream_t st, double* rec, const double* rec_init, long nrec_doubles, double* qt,
                           const double* qt_init, int nqt, double* ptab, const double* ptab_init, int nptab, double* dxp,
                           int ndxp, lh_ctrl* ctrl);
hipError_t lh_launch_ldlt_probe(const double* S, const double* b, int n, double* x, int solver, double tol, int max_it,
                                int* iters);
hipError_t lh_launch_mfma_probe(const double* A, const double* B, double* D);
hipError_t lh_read_stamps(unsigned long long* out, int n, int reset);
hipError_t lh_launch_frames(hipStream_t st, int n_frames, const int64_t* obs_ptr, const double* pose_in,
                            const double* pts, const double* uv, const uint8_t* flag_in, lh_params prm, double* res,
                            double* pose_out, uint8_t* flag_out, double* rchi2_out, int32_t* iters_out,
                            int32_t* inliers_out);
}

namespace {

enum { KC_LIN = 0, KC_REDUCE = 1, KC_CTRL = 2, KC_ALLREDUCE = 3, KC_INIT = 4, KC_N = 8 };
const char* kKernelNames[KC_N] = {"k_lin", "k_reduce", "k_ctrl", "allreduce", "k_lin_init", "", "", ""};

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipSuccess) n = std::max<size_t>(count, 1);
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// ---- Eigen quaternion <-> matrix (host copies of the formulas the kernels use) ----
void q_from_R(const double* R, double q[4]) {
#define M(i, j) R[3 * (i) + (j)]
    double t = M(0, 0) + M(1, 1) + M(2, 2);
    if (t > 0.0) {
        t = std::sqrt(t + 1.0);
        q[0] = 0.5 * t;
        t = 0.5 / t;
        q[1] = (M(2, 1) - M(1, 2)) * t;
        q[2] = (M(0, 2) - M(2, 0)) * t;
        q[3] = (M(1, 0) - M(0, 1)) * t;
    } else {
        int i = 0;
        if (M(1, 1) > M(0, 0)) i = 1;
        if (M(2, 2) > M(i, i)) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(M(i, i) - M(j, j) - M(k, k) + 1.0);
        double c[3];
        c[i] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (M(k, j) - M(j, k)) * t;
        c[j] = (M(j, i) + M(i, j)) * t;
        c[k] = (M(k, i) + M(i, k)) * t;
        q[1] = c[0]; q[2] = c[1]; q[3] = c[2];
    }
#undef M
}

void R_from_q(const double q[4], double R[9]) {
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;          R[2] = txz + twy;
    R[3] = txy + twz;          R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;          R[7] = tyz + twx;          R[8] = 1.0 - (txx + tyy);
}

void cross3(const double a[3], const double b[3], double c[3]) {
    const double c0 = a[1] * b[2] - a[2] * b[1], c1 = a[2] * b[0] - a[0] * b[2], c2 = a[0] * b[1] - a[1] * b[0];
    c[0] = c0; c[1] = c1; c[2] = c2;
}

void q_rotate(const double* q, const double v[3], double o[3]) {
    double uv[3], uv2[3];
    cross3(q + 1, v, uv);
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    cross3(q + 1, uv, uv2);
    for (int i = 0; i < 3; ++i) o[i] = v[i] + q[0] * uv[i] + uv2[i];
}

void q_mul(const double* a, const double* b, double o[4]) {
    double w = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    double x = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    double y = a[0] * b[2] + a[2] * b[0] + a[3] * b[1] - a[1] * b[3];
    double z = a[0] * b[3] + a[3] * b[0] + a[1] * b[2] - a[2] * b[1];
    const double sq = w * w + x * x + y * y + z * z;
    if (sq != 1.0) {
        const double sc = 2.0 / (1.0 + sq);
        w *= sc; x *= sc; y *= sc; z *= sc;
    }
    o[0] = w; o[1] = x; o[2] = y; o[3] = z;
}

// host mirror of d_pose_table (lh_kernels.hip): estimate_ -> (q_T, t_T, ext*T, R_T)
void pose_table(const double* T12, const double* e, double* pt) {
    const double R[9] = {T12[0], T12[1], T12[2], T12[4], T12[5], T12[6], T12[8], T12[9], T12[10]};
    double q[4];
    q_from_R(R, q);
    const double t[3] = {T12[3], T12[7], T12[11]};
    for (int i = 0; i < 4; ++i) pt[LH_PT_QT + i] = q[i];
    for (int i = 0; i < 3; ++i) pt[LH_PT_TT + i] = t[i];
    double qet[4], rt[3];
    q_mul(e, q, qet);
    q_rotate(e, t, rt);
    for (int i = 0; i < 4; ++i) pt[LH_PT_QET + i] = qet[i];
    for (int i = 0; i < 3; ++i) pt[LH_PT_TET + i] = e[4 + i] + rt[i];
    double Rt[9];
    R_from_q(q, Rt);
    for (int i = 0; i < 9; ++i) pt[LH_PT_RT + i] = Rt[i];
    pt[23] = 0.0;
}

}  // namespace

struct lh_handle {
    lh_options opt;
    int device = 0;
    hipStream_t stream = nullptr;
    ncclComm_t comm = nullptr;
    bool uploaded = false;

    // window (host copies needed to answer a solve)
    int P = 0, L = 0, L_act = 0, ncam = 1;
    int64_t O = 0;
    uint32_t fixed_mask = 0;
    lh_params prm{};
    std::vector<int32_t> lm_perm;      // landmark record slot -> window landmark (-1: padding)
    std::vector<int64_t> obs_perm;     // chunked obs -> window obs
    std::vector<double> lm_in;         // window input positions (landmarks with no edge keep them)
    int n_chunks = 0;
    int tgroup_begin[LH_TMAX + 2] = {0};
    lh_rs_layout LY{};

    // device buffers
    DevBuf<lh_chunk> d_chunks;
    DevBuf<lh_subbatch> d_sbs;
    DevBuf<uint32_t> d_meta, d_pair_ptr, d_items, d_rsmap;
    DevBuf<uint16_t> d_pair_pq;
    DevBuf<double> d_uv, d_rec, d_rec_init, d_ptab, d_ptab_init, d_qt, d_qt_init, d_ext, d_rho, d_slabs,
        d_rs_stage, d_rs_commit, d_maxd, d_dxp;
    DevBuf<lh_ctrl> d_ctrl;
    // frontend pose-only batch (lh_estimate_pose)
    DevBuf<int64_t> f_ptr;
    DevBuf<double> f_pose_in, f_pts, f_uv, f_res, f_pose_out, f_rchi2;
    DevBuf<uint8_t> f_flag_in, f_flag_out;
    DevBuf<int32_t> f_iters, f_inl;
    lh_ctrl* h_ctrl = nullptr;   // pinned
    int* h_done = nullptr;       // pinned, mapped: k_ctrl raises it when the LM loop stops
    int* d_done = nullptr;       // device alias of h_done

    // profiling
    struct PendingEv { int kc; int trial; hipEvent_t a, b; };
    std::vector<PendingEv> pending;   // profiled launches of the current solve
    int cur_trial = 0;                 // trial index being enqueued (0 = initial linearisation)
    std::vector<hipEvent_t> event_pool;
    size_t event_next = 0;
    int64_t launches[KC_N] = {0};
    double total_ms[KC_N] = {0};
};

namespace {

bool g_debug = getenv("LH_DEBUG") != nullptr;
bool g_event_sync = getenv("LH_EVENT_SYNC") != nullptr;   // A/B: the per-trial event scheme

#define HIPCHK(x)                                                                                        \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) {                                                                          \
            if (g_debug) fprintf(stderr, "lego_ba: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return LH_E_HIP;                                                                             \
        }                                                                                                \
    } while (0)

#define NCCLCHK(x)                                                                                       \
    do {                                                                                                 \
        ncclResult_t r_ = (x);                                                                           \
        if (r_ != ncclSuccess) {                                                                         \
            if (g_debug) fprintf(stderr, "lego_ba: %s failed: %s\n", #x, ncclGetErrorString(r_)); \
            return LH_E_RCCL;                                                                            \
        }                                                                                                \
    } while (0)

hipEvent_t next_event(lh_handle* h) {
    if (h->event_next == h->event_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        h->event_pool.push_back(e);
    }
    return h->event_pool[h->event_next++];
}

struct Prof {
    lh_handle* h;
    int kc;
    hipEvent_t a = nullptr, b = nullptr;
    Prof(lh_handle* hh, int k) : h(hh), kc(k) {
        if (h->opt.profile) {
            a = next_event(h);
            b = next_event(h);
            if (a) (void)hipEventRecord(a, h->stream);
        }
    }
    ~Prof() {
        if (a && b) {
            (void)hipEventRecord(b, h->stream);
            h->pending.push_back({kc, h->cur_trial, a, b});
        }
    }
};

// Launches enqueued for trials past the device's stop (trial > trials_run) exit at their first
// instruction; they are not counted as kernel work.
void collect_profile(lh_handle* h, int trials_run) {
    for (auto& pe : h->pending) {
        float ms = 0.f;
        if (pe.trial > trials_run) continue;
        if (hipEventElapsedTime(&ms, pe.a, pe.b) == hipSuccess) {
            h->launches[pe.kc] += 1;
            h->total_ms[pe.kc] += ms;
        }
    }
    h->pending.clear();
    h->event_next = 0;
}

int validate(const lh_window* w) {
    if (!w) return LH_E_BADARG;
    if (w->n_poses < 0 || w->n_landmarks < 0 || w->n_obs < 0) return LH_E_BADARG;
    if (w->n_poses > 0 && !w->pose_Tcw) return LH_E_BADARG;
    if (w->n_landmarks > 0 && !w->lm_xyz) return LH_E_BADARG;
    if (w->n_obs > 0 && (!w->obs_pose || !w->obs_lm || !w->obs_uv)) return LH_E_BADARG;
    if (w->n_cams < 0 || w->n_cams > LH_MAX_CAMS || (w->n_cams > 0 && !w->cam_ext)) return LH_E_BADARG;
    const int ncam = w->n_cams > 0 ? w->n_cams : 1;
    for (int64_t o = 0; o < w->n_obs; ++o) {
        if (w->obs_pose[o] >= (uint32_t)w->n_poses || w->obs_lm[o] >= (uint32_t)w->n_landmarks) return LH_E_BADARG;
        if (w->obs_cam && w->obs_cam[o] >= ncam) return LH_E_BADARG;
    }
    return LH_OK;
}

int upload_impl(lh_handle* h, const lh_window* w) {
    int st = validate(w);
    if (st != LH_OK) return st;
    h->uploaded = false;
    const int P = w->n_poses, L = w->n_landmarks;
    const int64_t O = w->n_obs;
    if (h->opt.world_size <= 1 && (O == 0 || (P + L) == 0)) return LH_E_EMPTY;   // problem.cpp:157-161
    if (P > LH_PMAX) return LH_E_UNSUPPORTED;
    const int ncam = w->n_cams > 0 ? w->n_cams : 1;
    h->P = P; h->L = L; h->O = O; h->ncam = ncam;
    h->fixed_mask = 0;
    if (w->pose_fixed)
        for (int p = 0; p < P; ++p)
            if (w->pose_fixed[p]) h->fixed_mask |= 1u << p;

    // ---- landmark-major CSR, observations in ascending pose order ----
    std::vector<int64_t> cnt(L + 1, 0);
    for (int64_t o = 0; o < O; ++o) cnt[w->obs_lm[o] + 1]++;
    for (int l = 0; l < L; ++l) cnt[l + 1] += cnt[l];
    std::vector<int64_t> csr(O);
    {
        std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
        for (int64_t o = 0; o < O; ++o) csr[pos[w->obs_lm[o]]++] = o;
    }
    std::vector<uint32_t> lm_mask(L, 0);
    std::vector<int> lm_first(L, 0), lm_last(L, 0);
    for (int l = 0; l < L; ++l) {
        auto b = csr.begin() + cnt[l], e = csr.begin() + cnt[l + 1];
        std::sort(b, e, [&](int64_t x, int64_t y) {
            if (w->obs_pose[x] != w->obs_pose[y]) return w->obs_pose[x] < w->obs_pose[y];
            return x < y;
        });
        uint32_t m = 0;
        for (auto it = b; it != e; ++it) {
            const uint32_t bit = 1u << w->obs_pose[*it];
            if (m & bit) return LH_E_UNSUPPORTED;   // two edges landmark->same pose (DESIGN.md "Limits")
            m |= bit;
        }
        if (e - b > LH_SB_OBS) return LH_E_UNSUPPORTED;
        if (__builtin_popcount(m) > LH_UMAX) return LH_E_UNSUPPORTED;
        lm_mask[l] = m;
        if (m) { lm_first[l] = __builtin_ctz(m); lm_last[l] = 31 - __builtin_clz(m); }
    }

    // ---- landmark order: by observation span, so chunks share small windows ----
    std::vector<int32_t> order;
    order.reserve(L);
    for (int l = 0; l < L; ++l)
        if (lm_mask[l]) order.push_back(l);   // landmarks without edges are not vertices (backend_lego.cpp:126)
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
        if (lm_first[a] != lm_first[b]) return lm_first[a] < lm_first[b];
        if (lm_last[a] != lm_last[b]) return lm_last[a] < lm_last[b];
        return lm_mask[a] < lm_mask[b];
    });
    const int Lact = (int)order.size();
    // ~512 chunks (2 workgroups per CU), 4*8-landmark multiples so the 4 waves get equal work
    int chunk_lm = (int)((Lact + 511) / 512);
    chunk_lm = ((chunk_lm + 4 * LH_SB_LM - 1) / (4 * LH_SB_LM)) * (4 * LH_SB_LM);
    chunk_lm = std::max(32, std::min(256, chunk_lm));
    if (const char* e = getenv("LH_CHUNK_LM")) {   // A/B knob for the chunk size (scripts/gpu_ab_chunk.sh)
        const int v = atoi(e);
        if (v >= LH_SB_LM && v <= 512) chunk_lm = v;
    }

    struct ChunkTmp { std::vector<int32_t> lms; uint32_t mask; };
    std::vector<ChunkTmp> ctmp;
    // a chunk's MFMA tile count T is set by the union of its landmarks' poses: start a new
    // chunk rather than let the union grow past the larger of the two tile counts
    auto chunkT = [](uint32_t mask) { return (6 * __builtin_popcount(mask) + 15) / 16; };
    for (int32_t l : order) {
        const uint32_t m = lm_mask[l];
        if (ctmp.empty() || (int)ctmp.back().lms.size() >= chunk_lm ||
            __builtin_popcount(ctmp.back().mask | m) > LH_UMAX ||
            chunkT(ctmp.back().mask | m) > std::max(chunkT(ctmp.back().mask), chunkT(m))) {
            ctmp.push_back(ChunkTmp{{}, 0u});
        }
        ctmp.back().lms.push_back(l);
        ctmp.back().mask |= m;
    }
    // group chunks by MFMA tile count T (one launch per T)
    std::vector<int> corder(ctmp.size());
    std::iota(corder.begin(), corder.end(), 0);
    std::stable_sort(corder.begin(), corder.end(), [&](int a, int b) { return chunkT(ctmp[a].mask) < chunkT(ctmp[b].mask); });

    std::vector<lh_chunk> chunks;
    std::vector<lh_subbatch> sbs;
    std::vector<uint32_t> meta;
    std::vector<double> uv, rec_init;
    h->lm_perm.clear();
    h->obs_perm.clear();
    for (int T = 0; T <= LH_TMAX + 1; ++T) h->tgroup_begin[T] = 0;
    int slot_of[32];
    auto pow2ceil = [](int k) { int g = 1, lg = 0; while (g < k) { g <<= 1; ++lg; } return lg; };
    for (int ci : corder) {
        const ChunkTmp& c = ctmp[ci];
        lh_chunk ck{};
        const int U = __builtin_popcount(c.mask);
        ck.U = (uint8_t)U;
        ck.T = (uint8_t)chunkT(c.mask);
        {
            int s = 0;
            for (int p = 0; p < 32; ++p) {
                if (c.mask & (1u << p)) { ck.pose[s] = (uint16_t)p; slot_of[p] = s; ++s; }
            }
        }
        ck.sb_begin = (uint32_t)sbs.size();
        // sub-batches: landmark l owns the aligned lane group [l*G, l*G + k_l) of 64 slots
        size_t i = 0;
        while (i < c.lms.size()) {
            int lg = 0, n = 0;
            while (i + n < c.lms.size() && n < LH_SB_LM) {
                const int32_t l = c.lms[i + n];
                const int lgn = std::max(lg, pow2ceil((int)(cnt[l + 1] - cnt[l])));
                if ((n + 1) << lgn > LH_SB_OBS) break;
                lg = lgn;
                ++n;
            }
            lh_subbatch sb{};
            sb.lm_begin = (uint32_t)(sbs.size() * LH_SB_LM);   // records sb*8 .. sb*8+7
            h->lm_perm.resize(sb.lm_begin + LH_SB_LM, -1);
            rec_init.resize((size_t)(sb.lm_begin + LH_SB_LM) * LH_REC, 0.0);
            sb.n_lm = (uint8_t)n;
            sb.lg = (uint8_t)lg;
            const size_t base = meta.size();
            meta.resize(base + LH_SB_OBS, 0u);
            uv.resize(2 * (base + LH_SB_OBS), 0.0);
            h->obs_perm.resize(base + LH_SB_OBS, -1);
            for (int q = 0; q < n; ++q) {
                const int32_t l = c.lms[i + q];
                h->lm_perm[sb.lm_begin + q] = l;
                for (int a = 0; a < 3; ++a) rec_init[(size_t)(sb.lm_begin + q) * LH_REC + LH_REC_X + a] = w->lm_xyz[3 * (size_t)l + a];
                int j = 0;
                for (int64_t r = cnt[l]; r < cnt[l + 1]; ++r, ++j) {
                    const int64_t o = csr[r];
                    const uint32_t p = w->obs_pose[o];
                    const uint32_t cam = w->obs_cam ? w->obs_cam[o] : 0;
                    const size_t slot = base + ((size_t)q << lg) + (size_t)j;
                    meta[slot] = LH_META(p, cam, slot_of[p], q);
                    uv[2 * slot] = w->obs_uv[2 * o];
                    uv[2 * slot + 1] = w->obs_uv[2 * o + 1];
                    h->obs_perm[slot] = o;
                }
            }
            sbs.push_back(sb);
            i += n;
        }
        ck.sb_end = (uint32_t)sbs.size();
        chunks.push_back(ck);
    }
    h->n_chunks = (int)chunks.size();
    // T group boundaries
    {
        int c = 0;
        for (int T = 1; T <= LH_TMAX + 1; ++T) {
            h->tgroup_begin[T] = c;
            while (c < h->n_chunks && chunks[c].T == T) ++c;
        }
        h->tgroup_begin[LH_TMAX + 1] = h->n_chunks;
        // a chunk window must fit one CU's LDS (a T = 6 window with 4 cameras does not)
        for (int T = 1; T <= LH_TMAX; ++T)
            if (h->tgroup_begin[T + 1] > h->tgroup_begin[T] && lh_lin_smem(T, ncam) > 160 * 1024) return LH_E_UNSUPPORTED;
    }

    // ---- reduce plan: for every pose pair (p <= q) the chunks touching it ----
    const int npairs = P * (P + 1) / 2;
    std::vector<uint16_t> pair_pq(2 * (size_t)std::max(npairs, 1));
    std::vector<std::vector<uint32_t>> plist(npairs);
    {
        int b = 0;
        for (int p = 0; p < P; ++p)
            for (int q = p; q < P; ++q, ++b) { pair_pq[2 * b] = (uint16_t)p; pair_pq[2 * b + 1] = (uint16_t)q; }
    }
    for (int ci = 0; ci < h->n_chunks; ++ci) {
        const lh_chunk& ck = chunks[ci];
        for (int s = 0; s < ck.U; ++s)
            for (int t = s; t < ck.U; ++t) {
                const int p = ck.pose[s], q = ck.pose[t];
                const int b = p * P - (p * (p - 1)) / 2 + (q - p);
                plist[b].push_back(((uint32_t)ci << 11) | ((uint32_t)ck.T << 8) | ((uint32_t)s << 4) | (uint32_t)t);
            }
    }
    std::vector<uint32_t> pair_ptr(npairs + 1, 0), items;
    for (int b = 0; b < npairs; ++b) {
        pair_ptr[b + 1] = pair_ptr[b] + (uint32_t)plist[b].size();
        items.insert(items.end(), plist[b].begin(), plist[b].end());
    }

    // ---- camera extrinsics (Sophus SE3 of Camera::pose_) and initial pose tables ----
    std::vector<double> ext(LH_EXT * (size_t)ncam);
    int ext_identity = 0;
    for (int c = 0; c < ncam; ++c) {
        static const double I12[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        const double* E = (w->n_cams > 0) ? w->cam_ext + 12 * c : I12;
        const double R[9] = {E[0], E[1], E[2], E[4], E[5], E[6], E[8], E[9], E[10]};
        double q[4], Rq[9];
        q_from_R(R, q);
        R_from_q(q, Rq);
        double* e = &ext[LH_EXT * (size_t)c];
        for (int i = 0; i < 4; ++i) e[i] = q[i];
        e[4] = E[3]; e[5] = E[7]; e[6] = E[11];
        for (int i = 0; i < 9; ++i) e[7 + i] = Rq[i];
        if (q[0] == 1.0 && q[1] == 0.0 && q[2] == 0.0 && q[3] == 0.0 && e[4] == 0.0 && e[5] == 0.0 && e[6] == 0.0)
            ext_identity |= 1 << c;
    }
    std::vector<double> pose(24 * (size_t)P), ptab(2 * (size_t)P * ncam * LH_PT);
    for (int p = 0; p < P; ++p) {
        const double* T = w->pose_Tcw + 12 * p;
        for (int s = 0; s < 2; ++s) {
            std::memcpy(&pose[12 * ((size_t)s * P + p)], T, 12 * sizeof(double));
            for (int c = 0; c < ncam; ++c)
                pose_table(T, &ext[LH_EXT * (size_t)c], &ptab[((size_t)s * P * ncam + (size_t)p * ncam + c) * LH_PT]);
        }
    }

    // ---- params ----
    lh_params& prm = h->prm;
    prm.P = P;
    prm.n = 6 * P;
    prm.ncam = ncam;
    prm.max_iters = h->opt.max_iters;
    prm.max_trials = h->opt.max_trials;
    prm.strategy = h->opt.strategy;
    prm.guard = h->opt.degenerate_guard;
    prm.lambda_given = h->opt.lambda_init >= 0.0;
    prm.ext_identity = ext_identity;
    prm.huber_delta = h->opt.huber_delta;
    prm.stop_dchi2 = h->opt.stop_dchi2;
    prm.tau = h->opt.tau;
    prm.lambda_cap = h->opt.lambda_cap;
    prm.lambda_init = h->opt.lambda_init;
    prm.solver = h->opt.linear_solver;
    prm.pcg_tol = h->opt.pcg_tol;
    prm.pcg_max_it = h->opt.pcg_max_iters;
    for (int i = 0; i < 4; ++i) prm.K[i] = w->K[i];
    h->LY = lh_rs_make(P);
    h->L_act = (int)h->lm_perm.size();   // landmark records (padded to 8 per sub-batch)
    // reduced-system element map for k_ctrl's register scatter: S element i of pose pair
    // (pi, pj), pi <= pj, row a, col b  ->  global rows gi = 6 pi + a, gj = 6 pj + b
    std::vector<uint32_t> rsmap((size_t)h->LY.npairs * 36);
    for (int pi = 0, blk = 0; pi < P; ++pi)
        for (int pj = pi; pj < P; ++pj, ++blk)
            for (int a = 0; a < 6; ++a)
                for (int b = 0; b < 6; ++b)
                    rsmap[(size_t)blk * 36 + 6 * a + b] = (uint32_t)(6 * pi + a) | ((uint32_t)(6 * pj + b) << 8) |
                                                        ((pi == pj ? 1u : 0u) << 16);
    h->lm_in.assign(w->lm_xyz, w->lm_xyz + 3 * (size_t)L);

    // ---- device buffers ----
    const size_t PT = (size_t)P * ncam * LH_PT;
    HIPCHK(h->d_chunks.ensure(chunks.size()));
    HIPCHK(h->d_sbs.ensure(sbs.size()));
    HIPCHK(h->d_meta.ensure(meta.size()));
    HIPCHK(h->d_uv.ensure(uv.size()));
    HIPCHK(h->d_pair_ptr.ensure(pair_ptr.size()));
    HIPCHK(h->d_items.ensure(items.size()));
    HIPCHK(h->d_pair_pq.ensure(pair_pq.size()));
    HIPCHK(h->d_rec_init.ensure(rec_init.size()));
    HIPCHK(h->d_rec.ensure(2 * rec_init.size()));
    HIPCHK(h->d_ptab.ensure(2 * PT));
    HIPCHK(h->d_ptab_init.ensure(2 * PT));
    HIPCHK(h->d_qt.ensure(pose.size()));
    HIPCHK(h->d_qt_init.ensure(pose.size()));
    HIPCHK(h->d_ext.ensure(ext.size()));
    HIPCHK(h->d_rho.ensure(meta.size()));
    HIPCHK(h->d_slabs.ensure((size_t)h->n_chunks * LH_SLAB_STRIDE));
    HIPCHK(h->d_rs_stage.ensure(h->LY.total));
    HIPCHK(h->d_rs_commit.ensure(h->LY.total));
    HIPCHK(h->d_rsmap.ensure(rsmap.size()));
    HIPCHK(h->d_maxd.ensure(1));
    HIPCHK(h->d_dxp.ensure(6 * (size_t)std::max(P, 1)));
    HIPCHK(h->d_ctrl.ensure(1));
    hipStream_t s = h->stream;
    auto up = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
        if (!bytes) return hipSuccess;
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s);
    };
    HIPCHK(up(h->d_chunks.p, chunks.data(), chunks.size() * sizeof(lh_chunk)));
    HIPCHK(up(h->d_sbs.p, sbs.data(), sbs.size() * sizeof(lh_subbatch)));
    HIPCHK(up(h->d_meta.p, meta.data(), meta.size() * sizeof(uint32_t)));
    HIPCHK(up(h->d_uv.p, uv.data(), uv.size() * sizeof(double)));
    HIPCHK(up(h->d_pair_ptr.p, pair_ptr.data(), pair_ptr.size() * sizeof(uint32_t)));
    HIPCHK(up(h->d_items.p, items.data(), items.size() * sizeof(uint32_t)));
    HIPCHK(up(h->d_pair_pq.p, pair_pq.data(), pair_pq.size() * sizeof(uint16_t)));
    HIPCHK(up(h->d_rec_init.p, rec_init.data(), rec_init.size() * sizeof(double)));
    HIPCHK(up(h->d_ptab_init.p, ptab.data(), ptab.size() * sizeof(double)));
    HIPCHK(up(h->d_qt_init.p, pose.data(), pose.size() * sizeof(double)));
    HIPCHK(up(h->d_ext.p, ext.data(), ext.size() * sizeof(double)));
    HIPCHK(up(h->d_rsmap.p, rsmap.data(), rsmap.size() * sizeof(uint32_t)));
    HIPCHK(hipStreamSynchronize(s));   // host vectors die at return
    h->uploaded = true;
    return LH_OK;
}

#define DBGSYNC(name)                                                                                   \
    do {                                                                                                \
        if (g_debug) {                                                                                  \
            hipError_t e_ = hipStreamSynchronize(s);                                                    \
            if (e_ == hipSuccess) e_ = hipGetLastError();                                               \
            if (e_ != hipSuccess) {                                                                     \
                fprintf(stderr, "lego_ba: %s failed: %s\n", name, hipGetErrorString(e_));               \
                return LH_E_HIP;                                                                        \
            }                                                                                           \
        }                                                                                               \
    } while (0)

int enqueue_trial(lh_handle* h, int mode) {
    hipStream_t s = h->stream;
    h->cur_trial = (mode == 0) ? 0 : h->cur_trial + 1;
    {
        Prof pr(h, mode == 0 ? KC_INIT : KC_LIN);
        for (int T = 1; T <= LH_TMAX; ++T) {
            const int c0 = h->tgroup_begin[T], c1 = h->tgroup_begin[T + 1];
            HIPCHK(lh_launch_lin(T, mode, c1 - c0, c0, s, h->d_chunks.p, h->d_sbs.p, h->d_uv.p,
                                 h->d_meta.p, h->d_rec.p, h->d_ptab.p, h->d_ext.p, h->d_ctrl.p, h->d_dxp.p,
                                 h->d_rho.p, h->d_slabs.p, h->prm, h->L_act, h->fixed_mask));
            DBGSYNC("k_lin");
        }
    }
    {
        Prof pr(h, KC_REDUCE);
        HIPCHK(lh_launch_reduce(s, h->d_chunks.p, h->d_slabs.p, h->d_pair_ptr.p, h->d_items.p, h->d_pair_pq.p,
                                h->d_ctrl.p, h->d_rs_stage.p, h->d_maxd.p, h->prm, h->n_chunks));
        DBGSYNC("k_reduce");
    }
    if (h->comm) {
        Prof pr(h, KC_ALLREDUCE);
        if (mode == 0) NCCLCHK(ncclAllReduce(h->d_maxd.p, h->d_maxd.p, 1, ncclFloat64, ncclMax, h->comm, s));
        NCCLCHK(ncclAllReduce(h->d_rs_stage.p, h->d_rs_stage.p, (size_t)h->LY.total, ncclFloat64, ncclSum, h->comm, s));
    }
    {
        Prof pr(h, KC_CTRL);
        HIPCHK(lh_launch_ctrl(s, h->d_ctrl.p, h->d_rs_commit.p, h->d_rs_stage.p, h->d_maxd.p, h->d_rsmap.p, h->d_qt.p, h->d_ptab.p,
                              h->d_ext.p, h->d_dxp.p, h->prm, mode, h->d_done, h->cur_trial));
        DBGSYNC("k_ctrl");
    }
    return LH_OK;
}

int solve_resident_impl(lh_handle* h, lh_result* out) {
    if (!h->uploaded) return LH_E_STATE;
    hipStream_t s = h->stream;
    const int P = h->P;
    const size_t PT = (size_t)P * h->ncam * LH_PT;
    // restart from the uploaded initial state (k_reset), then the LM trials.  Trials are
    // enqueued two ahead of the one the host waits for, so the device never idles on the
    // host; k_ctrl raises the mapped done flag and any trial enqueued after it is a no-op.
    hipEvent_t e0 = next_event(h), e1 = next_event(h);
    if (!e0 || !e1) return LH_E_HIP;
    volatile int* hd = h->h_done;   // [0] done, [1] last trial whose k_ctrl has started
    hd[0] = 0;
    hd[1] = -1;
    HIPCHK(hipEventRecord(e0, s));
    HIPCHK(lh_launch_reset(s, h->d_rec.p, h->d_rec_init.p, LH_REC * (long)h->L_act, h->d_qt.p, h->d_qt_init.p, 24 * P,
                           h->d_ptab.p, h->d_ptab_init.p, (int)(2 * PT), h->d_dxp.p, 6 * std::max(P, 1), h->d_ctrl.p));
    DBGSYNC("k_reset");
    int st = enqueue_trial(h, 0);
    if (st != LH_OK) return st;
    const int max_total = (h->opt.max_iters > 0) ? h->opt.max_iters * std::max(1, h->opt.max_trials) : 0;
    const int depth = h->opt.trials_per_sync > 0 ? std::min(h->opt.trials_per_sync, 32) : 2;
    int enq = 0;
    if (g_event_sync) {
        // previous scheme (A/B reference): one event per trial, host waits on the oldest
        hipEvent_t ring[64];
        int head = 0, tail = 0;
        auto push = [&]() -> int {
            int r = enqueue_trial(h, 1);
            if (r != LH_OK) return r;
            hipEvent_t ev = next_event(h);
            if (!ev) return LH_E_HIP;
            if (hipEventRecord(ev, s) != hipSuccess) return LH_E_HIP;
            ring[tail++ & 63] = ev;
            ++enq;
            return LH_OK;
        };
        while (enq < max_total && tail - head < depth)
            if ((st = push()) != LH_OK) return st;
        while (head < tail) {
            HIPCHK(hipEventSynchronize(ring[head++ & 63]));
            if (hd[0]) break;
            if (enq < max_total)
                if ((st = push()) != LH_OK) return st;
        }
    } else {
        // No per-trial events: k_ctrl writes the trial it starts into the mapped progress word,
        // and the host keeps `depth` trials enqueued past it until the device raises done.
        // hipStreamQuery every few thousand polls turns a device fault into an error return.
        unsigned spin = 0;
        while (!hd[0] && enq < max_total) {
            if (enq - hd[1] < depth) {
                if ((st = enqueue_trial(h, 1)) != LH_OK) return st;
                ++enq;
                continue;
            }
            if ((++spin & 4095) == 0) {
                const hipError_t q = hipStreamQuery(s);
                if (q != hipSuccess && q != hipErrorNotReady) return LH_E_HIP;
            }
            __builtin_ia32_pause();
        }
    }
    HIPCHK(hipEventRecord(e1, s));
    HIPCHK(hipMemcpyAsync(h->h_ctrl, h->d_ctrl.p, sizeof(lh_ctrl), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    const lh_ctrl& c = *h->h_ctrl;
    const int cur = c.cur;

    if (out) {
        out->iterations = c.iter;
        out->trials = c.trials;
        out->accepted = c.accepted;
        out->chi2_initial = c.chi2_initial;
        out->chi2_final = c.chi;
        out->lambda_final = c.lambda;
        out->time_ms = ms;
        out->pcg_iterations = c.pcg_iters;
        out->trace_len = std::min(c.trace_len, std::min(out->trace_cap, LH_TRACE));
        for (int i = 0; i < out->trace_len; ++i) {
            if (out->trace_chi2) out->trace_chi2[i] = c.trace_chi[i];
            if (out->trace_lambda) out->trace_lambda[i] = c.trace_lambda[i];
        }
        if (out->pose_Tcw && P)   // estimate_ of every VertexPose (backend_lego.cpp:198-213)
            HIPCHK(hipMemcpy(out->pose_Tcw, h->d_qt.p + 12 * (size_t)cur * P, 12 * (size_t)P * sizeof(double),
                             hipMemcpyDeviceToHost));
        if (out->lm_xyz) {
            std::memcpy(out->lm_xyz, h->lm_in.data(), h->lm_in.size() * sizeof(double));
            std::vector<double> R(LH_REC * (size_t)h->L_act);
            if (h->L_act)
                HIPCHK(hipMemcpy(R.data(), h->d_rec.p + LH_REC * (size_t)cur * h->L_act, R.size() * sizeof(double),
                                 hipMemcpyDeviceToHost));
            for (int i = 0; i < h->L_act; ++i)
                if (h->lm_perm[i] >= 0)
                    for (int a = 0; a < 3; ++a)
                        out->lm_xyz[3 * (size_t)h->lm_perm[i] + a] = R[LH_REC * (size_t)i + LH_REC_X + a];
        }
        if (out->edge_robust_chi2) {
            std::vector<double> r(h->obs_perm.size());
            if (!r.empty()) HIPCHK(hipMemcpy(r.data(), h->d_rho.p, r.size() * sizeof(double), hipMemcpyDeviceToHost));
            for (size_t i = 0; i < r.size(); ++i)
                if (h->obs_perm[i] >= 0) out->edge_robust_chi2[h->obs_perm[i]] = r[i];
        }
    }
    if (h->opt.verbose) {
        printf("==========LEGO OPTIMIZER (MI355X)==========\n");
        for (int i = 0; i < std::min(c.trace_len, LH_TRACE); ++i)
            printf("Iteration = %d,\tChi = %g,\tLambda = %g\n", i, c.trace_chi[i], c.trace_lambda[i]);
        printf("\nInfo: \nTimeCost(SolveProblem) = %g ms\n", (double)ms);
    }
    if (h->opt.profile) collect_profile(h, c.trials);
    else h->event_next = 0;
    return LH_OK;
}

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

const char* lh_strerror(int status) {
    switch (status) {
        case LH_OK: return "ok";
        case LH_E_EMPTY: return "empty problem: no vertices or no edges";
        case LH_E_BADARG: return "bad argument";
        case LH_E_HIP: return "HIP runtime error";
        case LH_E_RCCL: return "RCCL error";
        case LH_E_UNSUPPORTED: return "window outside the supported envelope";
        case LH_E_STATE: return "call out of order";
        default: return "unknown status";
    }
}

const char* lh_kernel_name(int kc) { return (kc >= 0 && kc < KC_N) ? kKernelNames[kc] : ""; }

void lh_default_options(lh_options* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->abi_version = LH_ABI_VERSION;
    o->max_iters = 10;
    o->max_trials = 10;
    o->strategy = LH_STRATEGY_DEFAULT;
    o->huber_delta = 5.991;
    o->stop_dchi2 = 1e-5;
    o->tau = 1e-5;
    o->lambda_cap = 5e10;
    o->lambda_init = -1.0;
    o->linear_solver = LH_SOLVER_LDLT;
    o->verbose = 0;
    o->device = -1;
    o->world_size = 1;
    o->rank = 0;
    o->degenerate_guard = 0;
    o->trials_per_sync = 0;
    o->profile = 0;
    o->pcg_max_iters = 0;
    o->pcg_tol = 1e-6;
}

int lh_comm_unique_id(uint8_t out[128]) {
    if (!out) return LH_E_BADARG;
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    std::memcpy(out, &id, 128);
    return LH_OK;
}

int lh_create(lh_handle** hp, const lh_options* opt) {
    if (!hp || !opt) return LH_E_BADARG;
    *hp = nullptr;
    if (opt->abi_version != LH_ABI_VERSION) return LH_E_BADARG;
    if (opt->max_iters < 0 || opt->max_trials < 0 || opt->world_size < 1 || opt->rank < 0 ||
        opt->rank >= opt->world_size || (opt->strategy != 0 && opt->strategy != 1))
        return LH_E_BADARG;
    if (opt->linear_solver != LH_SOLVER_LDLT && opt->linear_solver != LH_SOLVER_PCG) return LH_E_BADARG;
    if (opt->linear_solver == LH_SOLVER_PCG && !(opt->pcg_tol >= 0.0)) return LH_E_BADARG;
    lh_handle* h = new (std::nothrow) lh_handle();
    if (!h) return LH_E_HIP;
    h->opt = *opt;
    int dev = opt->device;
    if (dev < 0) {
        if (hipGetDevice(&dev) != hipSuccess) { delete h; return LH_E_HIP; }
    }
    if (hipSetDevice(dev) != hipSuccess) { delete h; return LH_E_HIP; }
    h->device = dev;
    if (lh_prepare_lin() != hipSuccess) { delete h; return LH_E_HIP; }
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) { delete h; return LH_E_HIP; }
    if (hipHostMalloc((void**)&h->h_ctrl, sizeof(lh_ctrl), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&h->h_done, 2 * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&h->d_done, h->h_done, 0) != hipSuccess) {
        lh_destroy(h);
        return LH_E_HIP;
    }
    // LH_FORCE_RCCL=1 builds a one-rank communicator on a single GPU, so the data-path
    // collectives (and their stream ordering) run in single-GPU tests too
    const char* force = std::getenv("LH_FORCE_RCCL");
    const bool force_comm = opt->world_size == 1 && force && force[0] == '1';
    if (opt->world_size > 1 || force_comm) {
        ncclUniqueId id;
        if (force_comm) {
            if (ncclGetUniqueId(&id) != ncclSuccess) { lh_destroy(h); return LH_E_RCCL; }
        } else {
            std::memcpy(&id, opt->comm_id, sizeof(id));
        }
        if (ncclCommInitRank(&h->comm, opt->world_size, id, opt->rank) != ncclSuccess) {
            h->comm = nullptr;
            lh_destroy(h);
            return LH_E_RCCL;
        }
    }
    *hp = h;
    return LH_OK;
}

void lh_destroy(lh_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->comm) ncclCommDestroy(h->comm);
    for (auto e : h->event_pool) (void)hipEventDestroy(e);
    h->f_ptr.release(); h->f_pose_in.release(); h->f_pts.release(); h->f_uv.release(); h->f_res.release();
    h->f_pose_out.release(); h->f_rchi2.release(); h->f_flag_in.release(); h->f_flag_out.release();
    h->f_iters.release(); h->f_inl.release();
    h->d_chunks.release(); h->d_sbs.release(); h->d_meta.release();
    h->d_pair_ptr.release(); h->d_items.release(); h->d_pair_pq.release();
    h->d_uv.release(); h->d_rec.release(); h->d_rec_init.release(); h->d_ptab.release();
    h->d_ptab_init.release(); h->d_qt.release(); h->d_qt_init.release(); h->d_ext.release(); h->d_rho.release();
    h->d_slabs.release(); h->d_rs_stage.release(); h->d_rs_commit.release(); h->d_rsmap.release(); h->d_maxd.release(); h->d_dxp.release();
    h->d_ctrl.release();
    if (h->h_ctrl) (void)hipHostFree(h->h_ctrl);
    if (h->h_done) (void)hipHostFree(h->h_done);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int lh_upload(lh_handle* h, const lh_window* in) {
    if (!h) return LH_E_BADARG;
    if (hipSetDevice(h->device) != hipSuccess) return LH_E_HIP;
    try {
        return upload_impl(h, in);
    } catch (const std::bad_alloc&) {
        return LH_E_HIP;
    } catch (...) {
        return LH_E_BADARG;
    }
}

int lh_solve_resident(lh_handle* h, lh_result* out) {
    if (!h) return LH_E_BADARG;
    if (hipSetDevice(h->device) != hipSuccess) return LH_E_HIP;
    try {
        return solve_resident_impl(h, out);
    } catch (...) {
        return LH_E_HIP;
    }
}

int lh_solve(lh_handle* h, const lh_window* in, lh_result* out) {
    int st = lh_upload(h, in);
    if (st != LH_OK) return st;
    return lh_solve_resident(h, out);
}

int lh_kernel_stats_get(lh_handle* h, lh_kernel_stats* out) {
    if (!h || !out) return LH_E_BADARG;
    for (int i = 0; i < KC_N; ++i) { out->launches[i] = h->launches[i]; out->total_ms[i] = h->total_ms[i]; }
    return LH_OK;
}

int lh_set_profiling(lh_handle* h, int on) {
    if (!h) return LH_E_BADARG;
    h->opt.profile = on ? 1 : 0;
    return LH_OK;
}

void lh_kernel_stats_reset(lh_handle* h) {
    if (!h) return;
    for (int i = 0; i < KC_N; ++i) { h->launches[i] = 0; h->total_ms[i] = 0.0; }
}

// Frontend::EstimateCurrentPose for a batch of frames (frontend_lego.cpp:157-250): upload, one
// k_frames launch (one workgroup per frame), download.
int lh_estimate_pose(lh_handle* h, const lh_frames* in, lh_frames_result* out) {
    if (!h || !in || !out) return LH_E_BADARG;
    const int F = in->n_frames;
    if (F < 0 || (F > 0 && (!in->obs_ptr || !in->pose_Tcw))) return LH_E_BADARG;
    if (F == 0) { out->time_ms = 0.0; return LH_OK; }
    if (in->obs_ptr[0] != 0) return LH_E_BADARG;
    for (int f = 0; f < F; ++f)
        if (in->obs_ptr[f + 1] < in->obs_ptr[f] || in->obs_ptr[f + 1] - in->obs_ptr[f] > (int64_t)INT32_MAX)
            return LH_E_BADARG;
    const int64_t O = in->obs_ptr[F];
    if (O > 0 && (!in->pts_w || !in->obs_uv)) return LH_E_BADARG;
    if (!out->pose_Tcw) return LH_E_BADARG;
    if (hipSetDevice(h->device) != hipSuccess) return LH_E_HIP;
    hipStream_t s = h->stream;
    HIPCHK(h->f_ptr.ensure(F + 1));
    HIPCHK(h->f_pose_in.ensure(12 * (size_t)F));
    HIPCHK(h->f_pose_out.ensure(12 * (size_t)F));
    HIPCHK(h->f_pts.ensure(3 * (size_t)O));
    HIPCHK(h->f_uv.ensure(2 * (size_t)O));
    HIPCHK(h->f_res.ensure(2 * (size_t)O));
    HIPCHK(h->f_rchi2.ensure((size_t)O));
    HIPCHK(h->f_flag_in.ensure((size_t)O));
    HIPCHK(h->f_flag_out.ensure((size_t)O));
    HIPCHK(h->f_iters.ensure((size_t)F));
    HIPCHK(h->f_inl.ensure((size_t)F));
    auto up = [&](void* d, const void* src, size_t bytes) { return hipMemcpyAsync(d, src, bytes, hipMemcpyHostToDevice, s); };
    HIPCHK(up(h->f_ptr.p, in->obs_ptr, sizeof(int64_t) * (F + 1)));
    HIPCHK(up(h->f_pose_in.p, in->pose_Tcw, sizeof(double) * 12 * (size_t)F));
    if (O > 0) {
        HIPCHK(up(h->f_pts.p, in->pts_w, sizeof(double) * 3 * (size_t)O));
        HIPCHK(up(h->f_uv.p, in->obs_uv, sizeof(double) * 2 * (size_t)O));
        if (in->is_outlier) HIPCHK(up(h->f_flag_in.p, in->is_outlier, (size_t)O));
    }
    lh_params prm{};
    prm.max_iters = h->opt.max_iters;
    prm.max_trials = h->opt.max_trials;
    prm.strategy = h->opt.strategy;
    prm.lambda_given = h->opt.lambda_init >= 0.0;
    prm.huber_delta = h->opt.huber_delta;
    prm.stop_dchi2 = h->opt.stop_dchi2;
    prm.tau = h->opt.tau;
    prm.lambda_cap = h->opt.lambda_cap;
    prm.lambda_init = h->opt.lambda_init;
    for (int i = 0; i < 4; ++i) prm.K[i] = in->K[i];
    hipEvent_t e0 = next_event(h), e1 = next_event(h);
    if (!e0 || !e1) return LH_E_HIP;
    HIPCHK(hipEventRecord(e0, s));
    HIPCHK(lh_launch_frames(s, F, h->f_ptr.p, h->f_pose_in.p, h->f_pts.p, h->f_uv.p,
                            in->is_outlier ? h->f_flag_in.p : nullptr, prm, h->f_res.p, h->f_pose_out.p,
                            h->f_flag_out.p, h->f_rchi2.p, h->f_iters.p, h->f_inl.p));
    HIPCHK(hipEventRecord(e1, s));
    auto down = [&](void* dst, const void* d, size_t bytes) { return hipMemcpyAsync(dst, d, bytes, hipMemcpyDeviceToHost, s); };
    HIPCHK(down(out->pose_Tcw, h->f_pose_out.p, sizeof(double) * 12 * (size_t)F));
    if (out->is_outlier && O > 0) HIPCHK(down(out->is_outlier, h->f_flag_out.p, (size_t)O));
    if (out->edge_chi2 && O > 0) HIPCHK(down(out->edge_chi2, h->f_rchi2.p, sizeof(double) * (size_t)O));
    if (out->n_inliers) HIPCHK(down(out->n_inliers, h->f_inl.p, sizeof(int32_t) * (size_t)F));
    if (out->iterations) HIPCHK(down(out->iterations, h->f_iters.p, sizeof(int32_t) * (size_t)F));
    HIPCHK(hipStreamSynchronize(s));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    out->time_ms = ms;
    h->event_next = 0;
    return LH_OK;
}

int lh_classify_outliers(const double* rchi2, int64_t n_obs, double chi2_th, uint8_t* is_outlier, double* th_out,
                         int64_t* n_inlier, int64_t* n_outlier) {
    if (n_obs < 0 || (n_obs > 0 && !rchi2)) return LH_E_BADARG;
    // backend_lego.cpp:164-184
    int64_t cin = 0, cout = 0;
    int iteration = 0;
    while (iteration < 5) {
        cout = 0;
        cin = 0;
        for (int64_t i = 0; i < n_obs; ++i) {
            if (rchi2[i] > chi2_th) cout++;
            else cin++;
        }
        double ratio = cin / double(cin + cout);
        if (ratio > 0.5) break;
        chi2_th *= 2;
        iteration++;
    }
    // :186-194
    if (is_outlier)
        for (int64_t i = 0; i < n_obs; ++i) is_outlier[i] = rchi2[i] > chi2_th ? 1 : 0;
    if (th_out) *th_out = chi2_th;
    if (n_inlier) *n_inlier = cin;
    if (n_outlier) *n_outlier = cout;
    return LH_OK;
}

// diagnostic hook: per-phase wave-cycle totals of the -DLH_STAMPS build (zeros otherwise)
int lh_debug_stamps(unsigned long long* out, int n, int reset) {
    if (!out || n < 0) return LH_E_BADARG;
    return lh_read_stamps(out, n, reset) == hipSuccess ? LH_OK : LH_E_HIP;
}

// test hook: k_ctrl's reduced-system solve on a dense symmetric S, device pointers
int lh_debug_ldlt_probe(const double* S, const double* b, int n, double* x) {
    if (!S || !b || !x) return LH_E_BADARG;
    if (n < 1 || n > LH_NPAD) return LH_E_UNSUPPORTED;
    HIPCHK(lh_launch_ldlt_probe(S, b, n, x, 0, 0.0, 0, nullptr));
    HIPCHK(hipDeviceSynchronize());
    return LH_OK;
}

int lh_debug_pcg_probe(const double* S, const double* b, int n, double tol, int max_iters, double* x, int* iters) {
    if (!S || !b || !x || !(tol >= 0.0)) return LH_E_BADARG;
    if (n < 1 || n > LH_NPAD) return LH_E_UNSUPPORTED;
    int* d_it = nullptr;
    HIPCHK(hipMalloc(&d_it, sizeof(int)));
    hipError_t e = lh_launch_ldlt_probe(S, b, n, x, 1, tol, max_iters, d_it);
    int it = 0;
    if (e == hipSuccess) e = hipMemcpy(&it, d_it, sizeof(int), hipMemcpyDeviceToHost);
    (void)hipFree(d_it);
    if (e != hipSuccess) return LH_E_HIP;
    if (iters) *iters = it;
    return LH_OK;
}

// The per-kernel HIP-event bracket of lh_set_profiling includes the launch itself: this is the
// same bracket around an empty kernel on the handle's stream (mean of 64 after 8 warm-ups).
int lh_debug_event_floor(lh_handle* h, double* ms) {
    if (!h || !ms) return LH_E_BADARG;
    if (hipSetDevice(h->device) != hipSuccess) return LH_E_HIP;
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess) return LH_E_HIP;
    if (hipEventCreate(&b) != hipSuccess) { (void)hipEventDestroy(a); return LH_E_HIP; }
    double tot = 0.0;
    int st = LH_OK;
    for (int i = 0; i < 72 && st == LH_OK; ++i) {
        if (hipEventRecord(a, h->stream) != hipSuccess || lh_launch_nop(h->stream) != hipSuccess ||
            hipEventRecord(b, h->stream) != hipSuccess || hipEventSynchronize(b) != hipSuccess) {
            st = LH_E_HIP;
            break;
        }
        float e = 0.f;
        if (hipEventElapsedTime(&e, a, b) != hipSuccess) st = LH_E_HIP;
        if (i >= 8) tot += e;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (st == LH_OK) *ms = tot / 64.0;
    return st;
}

int lh_debug_mfma_probe(const double* A, const double* B, double* D) {
    if (lh_launch_mfma_probe(A, B, D) != hipSuccess) return LH_E_HIP;
    if (hipDeviceSynchronize() != hipSuccess) return LH_E_HIP;
    return LH_OK;
}

}  // extern "C"

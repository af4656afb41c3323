// lh_host.cpp — C ABI (include/lego_ba.h) of the MI355X BA solver: device buffers, the upload of
// a window (lh_plan.cpp preprocessing into pinned staging, one async copy per array), the LM launch
// loop, the per-trial exchange of a landmark-sharded solve, and the download of the results.
//
// Per solve nothing but kernel launches happens on the host: the whole LM loop (accept/reject,
// lambda schedule, stop rule) runs on the device, and the host keeps `depth` trials enqueued ahead
// of the device's progress word.  With >1 rank each trial carries one all-reduce of the packed
// reduced pose system; every rank issues exactly the same number of them (see solve_resident_impl).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/lego_ba.h"
#include "lh_common.h"
#include "lh_lk.h"
#include "lh_plan.h"

extern "C" {
hipError_t lh_prepare_lin(int lds_limit);
size_t lh_lin_smem(int T, int ncam);
hipError_t lh_launch_nop(hipStream_t st);
hipError_t lh_launch_outliers(hipStream_t st, const double* rho, const int32_t* obs_perm, long nslots, long n_obs,
                              double th0, unsigned* part, uint8_t* flags);
hipError_t lh_launch_p2p(hipStream_t st, double* rs, double* maxd, int n, lh_peers peers, int rank, int world,
                         int parity, unsigned long long tag, long slot, int mode, int* err);
hipError_t lh_launch_outlier_counts(hipStream_t st, const double* rho, const int32_t* obs_perm, long nslots, long n_obs,
                                    double th0, unsigned* part, double* tot);
hipError_t lh_launch_outlier_flags(hipStream_t st, const double* rho, const int32_t* obs_perm, long nslots, long n_obs,
                                   double th0, const double* gtot, uint8_t* flags);
hipError_t lh_launch_lin(int T, int trial, int nchunks, int chunk_base, hipStream_t st, const lh_chunk* chunks,
                         const lh_subbatch* sbs, const float* obs_uv, const uint32_t* obs_meta, double* rec,
                         double* ptab, const double* ext, const lh_ctrl* ctrl, const double* dxp,
                         double* edge_rho, double* rows, double* csc, const uint32_t* crow, uint8_t* wflag,
                         long nslots, lh_params prm, int nrec, const uint64_t* fixed_bits, double* pose_mat,
                         int writer, lh_reset_args rst);
hipError_t lh_launch_reduce(hipStream_t st, const double* rows, const double* csc, const uint32_t* red_tab, int nred,
                            lh_ctrl* ctrl, double* rs_stage, double* rs_commit, double* maxd,
                            lh_params prm, int n_chunks, int mode, int* host_done, int seq, double* img);
hipError_t lh_launch_img_init(hipStream_t st, double* img, int n);
hipError_t lh_launch_ldlt_g_probe(const double* S, const double* b, int n, double* x, double* gA);
hipError_t lh_launch_ctrl(hipStream_t st, lh_ctrl* ctrl, double* rs_commit, const double* rs_stage, const double* maxd,
                          const uint32_t* rsmap, const uint16_t* pair_pq, double* dxp, lh_params prm, int mode,
                          int* host_done, int seq, double* gA, const double* gS,
                          const int32_t* brow_ptr, const uint32_t* brow_ent, const uint16_t* units, lh_band_args band,
                          double* img);
hipError_t lh_launch_dense(hipStream_t st, const double* rs_stage, const uint16_t* pair_pq, const lh_ctrl* ctrl,
                           double* gS, int P);
hipError_t lh_launch_gather(hipStream_t st, const lh_ctrl* ctrl, const double* rec, const int32_t* lm_perm, int nrec,
                            const double* rho, const int32_t* obs_perm, long nslots, double* out_xyz, double* out_rho);
hipError_t lh_launch_ldlt_probe(const double* S, const double* b, int n, double* x, int solver, double tol, int max_it,
                                int* iters);
hipError_t lh_launch_mfma_probe(const double* A, const double* B, double* D);
hipError_t lh_read_stamps(unsigned long long* out, int n, int reset);
hipError_t lh_launch_lk_pyr(hipStream_t st, const uint8_t* src, int sw, int sh, int64_t sstep, uint8_t* dst, int dw,
                            int dh);
hipError_t lh_launch_lk_track(hipStream_t st, const lh_lk_levels* L1, const lh_lk_levels* L2, int levels, int n,
                              const float* kp1, const float* kp2_in, float* kp2_out, uint8_t* success, int inverse,
                              int has_initial);
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
        const size_t c = std::max<size_t>(count, 1);
        hipError_t e = hipMalloc(&p, c * sizeof(T));
        if (e == hipSuccess) n = c;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// pinned host staging, grown on demand and reused across windows
// A typed window into an arena (no ownership): the per-window tables share one device and one pinned
// allocation so they cross the link as one copy (upload_impl)
template <typename T>
struct View {
    T* p = nullptr;
    size_t n = 0;
    void release() { p = nullptr; n = 0; }
};
template <typename T>
struct HostBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        const size_t c = std::max<size_t>(count + count / 4, 1);   // headroom: the next window is similar
        hipError_t e = hipHostMalloc((void**)&p, c * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) n = c;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
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

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Planner threads: the CPUs this process may use (affinity mask, capped by a cgroup v2 CPU quota:
// a GPU box exposes every host core but grants a share of them), at most 16.
int auto_host_threads() {
    cpu_set_t set;
    int n = 8;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long per = 0;
        if (std::fscanf(f, "%31s %ld", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0) {
            const long quota = std::atol(q);
            if (quota > 0) n = std::min<long>(n, (quota + per - 1) / per);
        }
        std::fclose(f);
    }
    // the planner's passes are memory-bound and their pool meets at a barrier per pass; its workers are
    // pinned to the caller's last-level cache (lh_plan.cpp Pool), which has 8 cores on an EPYC 9575F.
    // C3 lh_solve on such a box with a 16-CPU quota: 2.12 ms at 8 threads, 2.18 at 12, 2.16 at 16
    // (unpinned: 3.55, 3.45, 2.69)
    return std::max(1, std::min(8, n));
}

}  // namespace

struct lh_handle {
    lh_options opt;
    int device = 0;
    int lds_limit = 160 * 1024;   // hipDeviceAttributeMaxSharedMemoryPerBlock of the device
    hipStream_t stream = nullptr;
    ncclComm_t comm = nullptr;
    bool host_comm = false;       // LH_COMM_HOST with world_size > 1
    bool p2p = false;             // LH_COMM_P2P with world_size > 1 (the caller's all-reduce carries the rest)
    DevBuf<double> d_xchg;        // P2P: this rank's exchange buffer (lh_common.h), IPC-exported
    lh_peers peers{};             // every rank's exchange buffer as mapped here (opened IPC handles)
    long xchg_slot = 0;           // doubles per slot
    uint32_t solve_gen = 0;       // P2P tags: solves so far (the same count on every rank)
    int* h_xerr = nullptr;        // P2P: host-mapped failure word (a peer's tag did not arrive)
    int* d_xerr = nullptr;
    bool uploaded = false;
    bool upload_joined = false;   // this upload has taken part in the sharded envelope all-reduce
    bool upload_tail = false;     // ... and every rank passed it: the upload's closing status all-reduce follows
    lh::Pool* pool = nullptr;

    // window
    lh::Plan plan;
    int P = 0, L = 0, ncam = 1, n_rec = 0;
    int64_t O = 0, n_slots = 0;
    lh_params prm{};
    lh_rs_layout LY{};
    double last_prep_ms = 0.0, last_upload_ms = 0.0;

    // pinned staging of the upload
    View<lh_chunk> s_chunks;                                  // the per-window tables: views into s_arena
    View<lh_subbatch> s_sbs;
    View<uint32_t> s_items, s_pair_ptr, s_rsmap, s_brow_ent, s_red;
    View<uint16_t> s_pair_pq;
    View<uint16_t> s_units;                                   // k_ctrl's work units (lh_ctrl_units)
    View<uint16_t> s_bunits;                                  // k_ctrl_b's work units
    View<int32_t> s_bblk;                                     // k_ctrl_b's pair -> block table
    View<int32_t> s_lm_perm, s_brow_ptr;
    View<uint64_t> s_fixed;
    View<double> s_qt, s_ptab, s_ext;
    HostBuf<uint8_t> s_arena;
    size_t arena_bytes = 0;
    HostBuf<uint32_t> s_meta;
    HostBuf<int32_t> s_obs_perm;
    HostBuf<float> s_uv;                                     // pixels, 2 floats per slot
    HostBuf<double> s_lm, s_rs;                              // s_rs: the host-exchange buffer
    HostBuf<double> s_out;                                   // pinned staging of the download
    DevBuf<unsigned> d_ocnt;                                 // the outlier pass's per-block counts (ABI 5)
    DevBuf<uint8_t> d_oflag;                                 // its flags (window order), then threshold and counts
    DevBuf<double> d_otot;                                   // a sharded pass: this rank's counts, then all ranks' sums
    HostBuf<uint8_t> s_oflag;                                // pinned staging of the flags
    hipEvent_t ev_staging = nullptr;   // the upload's last copy out of the staging (reused by the next upload)
    bool staging_pending = false;

    // device buffers
    View<lh_chunk> d_chunks;                                  // the per-window tables: views into d_arena
    View<lh_subbatch> d_sbs;
    View<uint32_t> d_pair_ptr, d_items, d_rsmap, d_red;
    int n_red = 0;   // k_reduce's pair blocks (d_red: 4 words each, then the scalar block's sentinel)
    View<uint16_t> d_pair_pq, d_units, d_bunits;
    View<int32_t> d_bblk;
    DevBuf<double> d_band;        // k_ctrl_b: L rows (ceil16(6P) x 128) | ND per block (steps x 64), per ladder rung
    size_t lad_stride = 0;        // doubles of d_gA per ladder rung (k_ctrl_g, k_ctrl_p)
    bool band = false;            // this window's LDL^T runs in k_ctrl_b
    bool band_narrow = false;     // ... and every row's envelope starts within 56 rows of its 8-row block
    bool band_lu = false;         // ... and some step needs the stream loaders as unit waves too
    lh_ctrl_nd nd{};              // k_ctrl's two-chain schedule (nd.nsteps 0: the one-chain one)
    View<int32_t> d_lm_perm;
    View<double> d_ptab_init, d_qt_init, d_ext;
    DevBuf<uint8_t> d_arena;
    DevBuf<uint32_t> d_meta;
    DevBuf<int32_t> d_obs_perm;
    DevBuf<float> d_uv;
    DevBuf<double> d_lm_in, d_rec, d_ptab, d_qt, d_rho, d_rows, d_csc, d_gA, d_gS, d_rs_stage,
        d_rs_commit, d_maxd, d_dxp, d_out_xyz, d_out_rho;
    DevBuf<lh_ctrl> d_ctrl;
    View<uint64_t> d_fixed;      // fixed-pose bits (Plan::fixed_bits)
    View<int32_t> d_brow_ptr;    // the reduced system's block rows (Plan::brow_ptr / brow_ent, k_ctrl_p)
    View<uint32_t> d_brow_ent;
    DevBuf<uint8_t> d_wflag;     // [2][n_slots] inlier flags of each state buffer's linearisation (k_lin)
    DevBuf<double> d_img;        // [2][LH_IMG_SZ] k_ctrl's LDS system image, staged / committed (prm.img)
    // frontend pose-only batch (lh_estimate_pose)
    // inputs and outputs each packed into one arena, so a call is one upload and one download
    // through pinned staging (a single frame is latency-bound: every extra copy costs ~10 us)
    DevBuf<uint8_t> f_in, f_out;
    DevBuf<double> f_res;
    HostBuf<uint8_t> s_fin, s_fout;
    // LK optical flow (lh_lk_track): both images' pyramids, keypoints
    DevBuf<uint8_t> k_img[2], k_succ;
    DevBuf<float> k_kp1, k_kp2;
    lh_ctrl* h_ctrl = nullptr;   // pinned
    int last_chains = -1;        // lh_debug_chains: the last synchronous solve's stop chain
    int last_lskips = -1;        // lh_debug_ladder: its rejections onto a built ladder rung
    int last_batches = -1;       // lh_debug_batch: its batches of evaluate-only rungs
    int last_retrials[2] = {-1, -1};   // lh_debug_batch: their acceptances (re-run; re-run and stopping)
    size_t rho_off = 0;          // the last solve's per-edge rho0 "as last evaluated": its rung buffer in d_rho (a batch)
    int* h_done = nullptr;       // pinned, mapped lh_host_words: [0] k_ctrl raises it when the LM loop stops, [1] progress
                                 // word 2 * (last live trial) + (one iteration from max_iters)
    int* d_done = nullptr;       // device alias of h_done

    // per-solve bookkeeping
    int64_t n_coll = 0;          // data-path all-reduces of the last solve

    // profiling
    struct PendingEv { int kc; int trial; hipEvent_t a, b; };
    std::vector<PendingEv> pending;
    int cur_trial = 0;
    std::vector<hipEvent_t> event_pool;
    size_t event_next = 0;
    int64_t launches[KC_N] = {0};
    double total_ms[KC_N] = {0};
};

namespace {

bool g_debug = getenv("LH_DEBUG") != nullptr;

#define HIPCHK(x)                                                                                        \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) {                                                                          \
            if (g_debug) fprintf(stderr, "lego_ba: %s failed: %s\n", #x, hipGetErrorString(e_));       \
            return LH_E_HIP;                                                                             \
        }                                                                                                \
    } while (0)

#define NCCLCHK(x)                                                                                       \
    do {                                                                                                 \
        ncclResult_t r_ = (x);                                                                           \
        if (r_ != ncclSuccess) {                                                                         \
            if (g_debug) fprintf(stderr, "lego_ba: %s failed: %s\n", #x, ncclGetErrorString(r_));      \
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

// the planner's slot batches go to the device as soon as they are final (plan_fill's on_slots), so
// the copies of the largest arrays overlap the rest of the fill
struct SlotCopy {
    lh_handle* h;
    hipError_t err;
};
void copy_slots(void* user, int64_t s0, int64_t s1) {
    SlotCopy* c = static_cast<SlotCopy*>(user);
    lh_handle* h = c->h;
    if (c->err != hipSuccess || s1 <= s0) return;
    const size_t n = (size_t)(s1 - s0);
    hipStream_t st = h->stream;
    hipError_t e = hipMemcpyAsync(h->d_meta.p + s0, h->s_meta.p + s0, n * sizeof(uint32_t), hipMemcpyHostToDevice, st);
    if (e == hipSuccess)
        e = hipMemcpyAsync(h->d_uv.p + 2 * s0, h->s_uv.p + 2 * s0, 2 * n * sizeof(float), hipMemcpyHostToDevice, st);
    if (e == hipSuccess)
        e = hipMemcpyAsync(h->d_obs_perm.p + s0, h->s_obs_perm.p + s0, n * sizeof(int32_t), hipMemcpyHostToDevice, st);
    c->err = e;
}

// host copies between caller memory and pinned staging, in ~256 KB blocks over the planner's pool
struct ByteSeg { void* dst; const void* src; size_t n; };
void par_copy(lh_handle* h, const ByteSeg* seg, int nseg) {
    const size_t blk = 262144;
    size_t total = 0;
    for (int k = 0; k < nseg; ++k) total += (seg[k].dst && seg[k].src) ? seg[k].n : 0;
    if (total < 4 * blk) {   // waking the pool costs more than copying a small call's bytes
        for (int k = 0; k < nseg; ++k)
            if (seg[k].dst && seg[k].src && seg[k].n) std::memcpy(seg[k].dst, seg[k].src, seg[k].n);
        return;
    }
    std::vector<std::pair<int, size_t>> jobs;
    for (int k = 0; k < nseg; ++k)
        if (seg[k].dst && seg[k].src)
            for (size_t o = 0; o < seg[k].n; o += blk) jobs.emplace_back(k, o);
    auto job = [&](int j) {
        const ByteSeg& g = seg[jobs[j].first];
        const size_t o = jobs[j].second, c = std::min(blk, g.n - o);
        std::memcpy((uint8_t*)g.dst + o, (const uint8_t*)g.src + o, c);
    };
    if (h->pool && jobs.size() > 1) h->pool->run((int)jobs.size(), job);
    else for (int j = 0; j < (int)jobs.size(); ++j) job(j);
}

// Wait for an event by polling it: hipEventSynchronize measured ~2 ms for lh_upload's copies that the
// solve path (which polls) sees finish within ~0.3 ms of the planner: the runtime's blocking wait
// wakes the thread late.
hipError_t spin_wait(hipEvent_t ev) {
    for (;;) {
        const hipError_t q = hipEventQuery(ev);
        if (q != hipErrorNotReady) return q;
        for (int i = 0; i < 64; ++i) __builtin_ia32_pause();
    }
}

// sync: return only once the copies are done (lh_upload); lh_solve leaves them queued ahead of its
// kernels on the same stream.  Either way the next upload waits for them before it rewrites the staging.
int upload_body(lh_handle* h, const lh_window* w, bool sync);
int rank_max(lh_handle* h, double* buf, int n);
int p2p_setup(lh_handle* h);

// Every exit after the first copy out of the pinned staging is queued must leave ev_staging recorded
// behind it, or the next upload could rewrite (or reallocate) the staging while that DMA still reads
// it: the error returns (LH_E_UNSUPPORTED envelope checks, a failed HIP call) record it here.
//
// A sharded upload holds one collective, the MAX all-reduce of the envelope of S (upload_body).  A rank that fails before it (a bad pixel, an unsupported window, an allocation)
// still joins it, contributing its status in word 0 and nothing to the envelope, so the healthy ranks
// are not left blocked in it: every rank then returns the largest status of any rank.
//
// A rank can also fail after that collective (the controllers' buffers, the image initialisation, the arena
// copy), when its peers have already passed it: so every rank that passed it (all of them, or none: the
// collective's status word is shared) closes the upload with a second MAX all-reduce of its final status, and
// a rank whose tail failed takes the others down with it instead of leaving them in the first trial's exchange.
int upload_impl(lh_handle* h, const lh_window* w, bool sync) {
    h->upload_joined = false;
    h->upload_tail = false;
    int st = upload_body(h, w, sync);
    const bool sharded = h->host_comm || h->comm || h->p2p;
    if (st != LH_OK && sharded && !h->upload_joined && w && w->n_poses > 0 && w->n_poses <= LH_PMAX_ANY) {
        std::vector<double> buf(1 + (size_t)w->n_poses, -1e300);
        buf[0] = (double)st;
        rank_max(h, buf.data(), 1 + w->n_poses);
    }
    if (sharded && h->upload_tail) {
        double fs = (double)st;
        const int st_r = rank_max(h, &fs, 1);
        if (st == LH_OK) st = (st_r != LH_OK) ? st_r : (int)fs;
        if (st != LH_OK) h->uploaded = false;
    }
    // the peer-write exchange's buffers once every rank's upload is through (its collectives run on all ranks)
    if (st == LH_OK && h->p2p) {
        st = p2p_setup(h);
        if (st != LH_OK) h->uploaded = false;
    }
    if (st != LH_OK && !h->staging_pending && h->ev_staging) {
        if (hipEventRecord(h->ev_staging, h->stream) == hipSuccess) h->staging_pending = true;
    }
    return st;
}

int upload_body(lh_handle* h, const lh_window* w, bool sync) {
    const double t0 = now_ms();
    h->uploaded = false;
    if (h->staging_pending) {
        HIPCHK(spin_wait(h->ev_staging));
        h->staging_pending = false;
    }
    // the landmark positions need no plan: they go out first and cross the link while the planner runs
    if (w && w->n_landmarks > 0 && w->lm_xyz) {
        const size_t nl = 3 * (size_t)w->n_landmarks;
        HIPCHK(h->d_lm_in.ensure(nl));
        HIPCHK(h->s_lm.ensure(nl));
        const ByteSeg seg{h->s_lm.p, w->lm_xyz, nl * sizeof(double)};
        par_copy(h, &seg, 1);
        HIPCHK(hipMemcpyAsync(h->d_lm_in.p, h->s_lm.p, nl * sizeof(double), hipMemcpyHostToDevice, h->stream));
    }
    lh::PlanCfg cfg;
    cfg.chunk_lm = h->opt.chunk_landmarks;
    lh::Plan& pl = h->plan;
    const bool sharded = h->host_comm || h->comm || h->p2p;
    cfg.rank_invariant_pairs = h->opt.world_size > 1;
    int st = lh::plan_structure(w, cfg, h->opt.world_size > 1, pl, h->pool);
    if (st != LH_OK) {
        HIPCHK(hipEventRecord(h->ev_staging, h->stream));
        h->staging_pending = true;
        return st;
    }
    // Pose p's first coupled pose: the lowest pose of any chunk window holding p (a chunk writes a block
    // for every pair of its window).  It gives the envelope of S in natural pose order, from which k_ctrl's
    // and k_ctrl_b's work units and the banded controller's eligibility follow; a sharded solve factors
    // the sum of every rank's blocks, so it takes the union over the ranks (below, after every rank-local
    // failure point).
    std::vector<int> pf(pl.P);
    for (int p = 0; p < pl.P; ++p) pf[p] = p;
    for (size_t c = 0; c < pl.chunk_mask.size(); ++c) {
        const uint64_t m = pl.chunk_mask[c];
        if (!m) continue;
        const int lo = pl.chunk_base[c] + __builtin_ctzll(m);
        for (uint64_t b = m; b; b &= b - 1) {
            const int p = pl.chunk_base[c] + __builtin_ctzll(b);
            pf[p] = std::min(pf[p], lo);
        }
    }
    // past LH_PMAX poses: LDL^T by k_ctrl_b when the reduced system is banded in natural pose order
    // (any P up to LH_PMAX_ANY), else by k_ctrl_g (dense, up to LH_PMAX_WIN poses); PCG by k_ctrl_p
    // (block-sparse, up to LH_PMAX_ANY).  Decided after the union below; the arena reserves the band's
    // tables whenever it may run.
    static const int kBandSteps = 6 * LH_PMAX_ANY / 8;
    const bool band_possible = pl.P > LH_PMAX && h->opt.linear_solver == LH_SOLVER_LDLT && !getenv("LH_NO_BAND");
    h->band = false;
    h->band_narrow = false;
    h->band_lu = false;
    // k_lin's write-through record stores address both record buffers through one buffer descriptor
    // (32-bit byte offsets): up to ~8.3 M landmarks per rank
    if ((size_t)2 * pl.n_rec * LH_REC * sizeof(double) > (size_t)INT32_MAX) return LH_E_UNSUPPORTED;
    // a chunk window must fit one CU's LDS
    for (int T = 1; T <= LH_TMAX; ++T)
        if (pl.tgroup_begin[T + 1] > pl.tgroup_begin[T] && lh_lin_smem(T, pl.ncam) > (size_t)h->lds_limit)
            return LH_E_UNSUPPORTED;
    const int P = pl.P, ncam = pl.ncam;
    h->P = P; h->L = pl.L; h->O = pl.O; h->ncam = ncam;
    h->n_rec = pl.n_rec;
    h->n_slots = pl.n_slots;
    h->LY = lh_rs_make(P, pl.npairs);

    // ---- device buffers (before the fill: its slot batches are copied as they complete) ----
    const size_t PT = (size_t)P * ncam * LH_PT;
    // The per-window tables (all but the observation slots and the positions) live in one arena, on the
    // device and in pinned staging, at the same offsets: they cross the link as one copy.  Each
    // hipMemcpyAsync costs ~10 us of DMA-engine turnaround beside its transfer (rocprofv3 memory-copy
    // trace of lh_upload), and the 13 small copies these were made most of the upload's tail.
    {
        size_t bytes = 0;
        auto part = [&](size_t b) { const size_t o = bytes; bytes += (b + 255) & ~(size_t)255; return o; };
        const size_t o_chunks = part(pl.n_chunks * sizeof(lh_chunk)), o_sbs = part((size_t)pl.n_sb * sizeof(lh_subbatch));
        const size_t o_lmp = part((size_t)pl.n_rec * sizeof(int32_t)), o_pptr = part(((size_t)pl.npairs + 1) * sizeof(uint32_t));
        const size_t o_items = part((size_t)pl.n_items * sizeof(uint32_t)), o_ppq = part(2 * (size_t)pl.npairs * sizeof(uint16_t));
        const size_t o_rsmap = part((size_t)pl.npairs * 36 * sizeof(uint32_t)), o_ptab = part(2 * PT * sizeof(double));
        const size_t o_qt = part(24 * (size_t)std::max(P, 1) * sizeof(double)), o_ext = part(LH_EXT * (size_t)ncam * sizeof(double));
        const size_t o_fix = part(pl.fixed_bits.size() * sizeof(uint64_t)), o_bptr = part(pl.brow_ptr.size() * sizeof(int32_t));
        const size_t o_bent = part(pl.brow_ent.size() * sizeof(uint32_t));
        const size_t o_units = part(16 * LH_NSTEP * sizeof(uint16_t));
        const size_t n_bunits = band_possible ? 16 * (size_t)kBandSteps : 0, n_bblk = band_possible ? (size_t)P * 64 : 0;
        const size_t o_bunits = part(n_bunits * sizeof(uint16_t));
        const size_t o_bblk = part(n_bblk * sizeof(int32_t));
        const size_t o_red = part(4 * ((size_t)pl.npairs + 1) * sizeof(uint32_t));
        HIPCHK(h->d_arena.ensure(bytes));
        HIPCHK(h->s_arena.ensure(bytes));
        h->arena_bytes = bytes;
        auto bind = [](auto& d, auto& st, uint8_t* dbase, uint8_t* sbase, size_t off, size_t count) {
            using T = std::remove_pointer_t<decltype(d.p)>;
            d.p = reinterpret_cast<T*>(dbase + off); d.n = count;
            st.p = reinterpret_cast<T*>(sbase + off); st.n = count;
        };
        uint8_t* db = h->d_arena.p;
        uint8_t* sb = h->s_arena.p;
        bind(h->d_chunks, h->s_chunks, db, sb, o_chunks, pl.n_chunks);
        bind(h->d_sbs, h->s_sbs, db, sb, o_sbs, pl.n_sb);
        bind(h->d_lm_perm, h->s_lm_perm, db, sb, o_lmp, pl.n_rec);
        bind(h->d_pair_ptr, h->s_pair_ptr, db, sb, o_pptr, pl.npairs + 1);
        bind(h->d_items, h->s_items, db, sb, o_items, pl.n_items);
        bind(h->d_pair_pq, h->s_pair_pq, db, sb, o_ppq, 2 * (size_t)pl.npairs);
        bind(h->d_rsmap, h->s_rsmap, db, sb, o_rsmap, (size_t)pl.npairs * 36);
        bind(h->d_ptab_init, h->s_ptab, db, sb, o_ptab, 2 * PT);
        bind(h->d_qt_init, h->s_qt, db, sb, o_qt, 24 * (size_t)std::max(P, 1));
        bind(h->d_ext, h->s_ext, db, sb, o_ext, LH_EXT * (size_t)ncam);
        bind(h->d_fixed, h->s_fixed, db, sb, o_fix, pl.fixed_bits.size());
        bind(h->d_brow_ptr, h->s_brow_ptr, db, sb, o_bptr, pl.brow_ptr.size());
        bind(h->d_brow_ent, h->s_brow_ent, db, sb, o_bent, pl.brow_ent.size());
        bind(h->d_units, h->s_units, db, sb, o_units, 16 * LH_NSTEP);
        bind(h->d_bunits, h->s_bunits, db, sb, o_bunits, n_bunits);
        bind(h->d_bblk, h->s_bblk, db, sb, o_bblk, n_bblk);
        bind(h->d_red, h->s_red, db, sb, o_red, 4 * ((size_t)pl.npairs + 1));
    }
    HIPCHK(h->d_meta.ensure(pl.n_slots));
    HIPCHK(h->d_uv.ensure(2 * pl.n_slots));
    HIPCHK(h->d_obs_perm.ensure(pl.n_slots));
    HIPCHK(h->d_lm_in.ensure(3 * (size_t)pl.L));
    HIPCHK(h->d_rec.ensure(2 * (size_t)pl.n_rec * LH_REC));
    HIPCHK(h->d_ptab.ensure(2 * PT));
    HIPCHK(h->d_qt.ensure(24 * (size_t)P));
    HIPCHK(h->d_wflag.ensure(2 * (size_t)pl.n_slots));
    HIPCHK(h->d_rows.ensure((size_t)pl.n_items * LH_ROW));
    HIPCHK(h->d_rs_stage.ensure(h->LY.total));
    HIPCHK(h->d_rs_commit.ensure(h->LY.total));
    // the lambda ladder's rungs, one controller workgroup each (LH_NO_LADDER=1: one rung, the A/B
    // switch): one pending step per rung, and per rung the controller's global scratch
    const int ladder = !getenv("LH_NO_LADDER") ? std::max(1, std::min(h->opt.max_trials, LH_LAD)) : 1;
    h->lad_stride = 0;
    if (P > LH_PMAX && h->opt.linear_solver == LH_SOLVER_PCG) {   // k_ctrl_p's row-contiguous copy of S (36 per block-row entry)
        h->lad_stride = pl.brow_ent.size() * 36;
        HIPCHK(h->d_gA.ensure((size_t)ladder * h->lad_stride));
    }
    HIPCHK(h->d_maxd.ensure(1));
    HIPCHK(h->d_dxp.ensure((size_t)ladder * 6 * (size_t)std::max(P, 1)));
    HIPCHK(h->d_ctrl.ensure(1));
    HIPCHK(h->d_out_xyz.ensure(3 * (size_t)pl.L));
    HIPCHK(h->d_out_rho.ensure(pl.O));
    if (h->host_comm) HIPCHK(h->s_rs.ensure(h->LY.total + 1));

    // ---- staging and the fill ----
    HIPCHK(h->s_meta.ensure(pl.n_slots));
    HIPCHK(h->s_uv.ensure(2 * pl.n_slots));
    HIPCHK(h->s_obs_perm.ensure(pl.n_slots));
    lh::PlanOut po{h->s_chunks.p, h->s_sbs.p, h->s_meta.p, h->s_uv.p, h->s_obs_perm.p, h->s_lm_perm.p,
                   h->s_items.p, h->s_pair_pq.p, h->s_rsmap.p, nullptr};   // positions: copied out above
    SlotCopy sc{h, hipSuccess};
    const int batches = pl.n_slots >= (1 << 16) ? 8 : 1;
    const int fs = lh::plan_fill(w, pl, po, h->pool, copy_slots, &sc, batches);
    HIPCHK(sc.err);
    if (fs != LH_OK) {   // a pixel that is not a float value; the slot copies already issued read the staging
        HIPCHK(hipEventRecord(h->ev_staging, h->stream));
        h->staging_pending = true;
        return fs;
    }
    std::memcpy(h->s_pair_ptr.p, pl.pair_ptr.data(), pl.pair_ptr.size() * sizeof(uint32_t));
    // k_reduce's blocks: one per pose pair that some chunk's rows reach ({block, first row, end row, p | q << 16}),
    // then the scalar block's sentinel.  One rank skips the pairs no chunk couples: their blocks of S are zero
    // for the whole window (the reduced-system buffers are cleared per window, below).  A sharded solve keeps
    // every pair: a rank's empty pair still has to write its zero contribution over last trial's all-reduced sum.
    {
        const bool skip = h->opt.world_size == 1 && !getenv("LH_NO_RED_SKIP");
        uint32_t* rt = h->s_red.p;
        int k = 0;
        for (int b = 0; b < pl.npairs; ++b) {
            const uint32_t ib = pl.pair_ptr[b], ie = pl.pair_ptr[b + 1];
            if (skip && ib == ie) continue;
            rt[4 * k] = (uint32_t)b; rt[4 * k + 1] = ib; rt[4 * k + 2] = ie;
            rt[4 * k + 3] = (uint32_t)pl.pair_list[2 * b] | ((uint32_t)pl.pair_list[2 * b + 1] << 16);
            ++k;
        }
        rt[4 * k] = (uint32_t)pl.npairs; rt[4 * k + 1] = 0; rt[4 * k + 2] = 0; rt[4 * k + 3] = 0;
        h->n_red = k;
        if (skip) {   // the skipped pairs' blocks (and every buffer slot k_reduce never writes) read as zero
            HIPCHK(hipMemsetAsync(h->d_rs_stage.p, 0, h->LY.total * sizeof(double), h->stream));
            HIPCHK(hipMemsetAsync(h->d_rs_commit.p, 0, h->LY.total * sizeof(double), h->stream));
        }
    }
    std::memcpy(h->s_fixed.p, pl.fixed_bits.data(), pl.fixed_bits.size() * sizeof(uint64_t));
    std::memcpy(h->s_brow_ptr.p, pl.brow_ptr.data(), pl.brow_ptr.size() * sizeof(int32_t));
    std::memcpy(h->s_brow_ent.p, pl.brow_ent.data(), pl.brow_ent.size() * sizeof(uint32_t));

    // ---- camera extrinsics (Sophus SE3 of Camera::pose_) and the initial pose tables ----
    double* ext = h->s_ext.p;
    int ext_identity = 0, ext_rot_identity = 0;
    for (int c = 0; c < ncam; ++c) {
        static const double I12[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        const double* E = (w->n_cams > 0) ? w->cam_ext + 12 * c : I12;
        const double R[9] = {E[0], E[1], E[2], E[4], E[5], E[6], E[8], E[9], E[10]};
        double q[4], Rq[9];
        q_from_R(R, q);
        R_from_q(q, Rq);
        double* e = ext + LH_EXT * (size_t)c;
        for (int i = 0; i < 4; ++i) e[i] = q[i];
        e[4] = E[3]; e[5] = E[7]; e[6] = E[11];
        for (int i = 0; i < 9; ++i) e[7 + i] = Rq[i];
        if (q[0] == 1.0 && q[1] == 0.0 && q[2] == 0.0 && q[3] == 0.0) {
            ext_rot_identity |= 1 << c;
            if (e[4] == 0.0 && e[5] == 0.0 && e[6] == 0.0) ext_identity |= 1 << c;
        }
    }
    for (int p = 0; p < P; ++p) {
        const double* T = w->pose_Tcw + 12 * p;
        for (int s = 0; s < 2; ++s) {
            std::memcpy(h->s_qt.p + 12 * ((size_t)s * P + p), T, 12 * sizeof(double));
            for (int c = 0; c < ncam; ++c)
                pose_table(T, ext + LH_EXT * (size_t)c, h->s_ptab.p + ((size_t)s * P * ncam + (size_t)p * ncam + c) * LH_PT);
        }
    }

    // ---- the sharded upload's envelope collective.  Word 0 carries the largest status of any rank (a rank
    //      that failed earlier joins from upload_impl with its own), then -pf per pose: the union envelope.
    //      Everything after it is decided on data identical on every rank; a rank-local failure after it
    //      (allocations, the image initialisation, the copies) is shared by upload_impl's closing status
    //      all-reduce. ----
    if (sharded) {
        std::vector<double> neg(1 + (size_t)P);
        neg[0] = 0.0;
        for (int p = 0; p < P; ++p) neg[1 + p] = -(double)pf[p];
        h->upload_joined = true;
        const int st_r = rank_max(h, neg.data(), 1 + P);
        if (st_r != LH_OK) return st_r;
        if (neg[0] > 0.0) return (int)neg[0];
        for (int p = 0; p < P; ++p) pf[p] = (int)(-neg[1 + p]);
        h->upload_tail = true;
        // (test hook) this rank fails after the collective, as a failed allocation in the tail would
        const char* fail_env = getenv("LH_TEST_FAIL_AFTER_ENVELOPE");
        if (fail_env && atoi(fail_env) == h->opt.rank) return LH_E_HIP;
    }

    // ---- the banded controller's eligibility (tile rows enter its window two steps before use) ----
    std::vector<uint16_t> bunits;
    if (band_possible) {
        const int n = 6 * P, NE = (n + 15) & ~15, NT = NE / 16;
        std::vector<int32_t> fcb(NT);
        bool ok = true;
        for (int I = 0; I < NT; ++I) {
            int f = 1 << 20;
            for (int r = 16 * I; r < 16 * I + 16; ++r) f = std::min(f, r < n ? 6 * pf[r / 6] : r);
            fcb[I] = f >> 3;
            if (I >= 8 && fcb[I] < 2 * I - 13) ok = false;   // a tile row must enter the window before it is used
        }
        if (ok) {
            bunits.resize(16 * (size_t)kBandSteps);
            const int order[LH_BAND_UNIT_WAVES] = LH_ORDER_BAND;
            // the 11 unit waves when every step fits them (k_ctrl_b<false>), else with the loaders too
            const int w11 = lh_ctrl_units(n, fcb.data(), order, 11, kBandSteps, bunits.data());
            h->band_lu = w11 > 11;
            if (h->band_lu)
                ok = lh_ctrl_units(n, fcb.data(), order, LH_BAND_UNIT_WAVES, kBandSteps, bunits.data()) <= LH_BAND_UNIT_WAVES;
        }
        h->band = ok;
        // k_ctrl_b's one-row-per-lane back substitution: block KB's L rows reach no column below KB - 56
        bool narrow = ok && !getenv("LH_NO_NARROW");
        for (int r = 0; r < n && narrow; ++r) narrow = 6 * pf[r / 6] >= (r & ~7) - 56;
        h->band_narrow = narrow;
    }
    if (P > LH_PMAX_WIN && h->opt.linear_solver == LH_SOLVER_LDLT && !h->band) return LH_E_UNSUPPORTED;
    // batches of evaluate-only rungs (every controller, one rank or sharded; LH_NO_BATCH=1: one rung
    // per chain, the A/B switch; LH_BATCH_MAX caps the rungs per batch): per rung a per-edge rho0 and the chunk scalars
    const bool dec1 = (P <= LH_PMAX || h->band) && h->opt.world_size == 1 && !h->comm;
    int batch = (ladder > 1 && !getenv("LH_NO_BATCH")) ? ladder : 1;
    if (const char* bm = getenv("LH_BATCH_MAX")) batch = std::max(1, std::min(batch, atoi(bm)));
    HIPCHK(h->d_rho.ensure((size_t)batch * pl.n_slots));
    HIPCHK(h->d_csc.ensure((size_t)batch * pl.n_chunks * 4));
    if (h->band) {   // k_ctrl_b's L rows and ND blocks; L entries outside the envelope are never written: zero
        const size_t NE = (size_t)((6 * P + 15) & ~15);
        const size_t per = NE * 128 + (size_t)(6 * LH_PMAX_ANY / 8) * 64;   // one rung's (k_ctrl_b's layout)
        HIPCHK(h->d_band.ensure((size_t)ladder * per));
        HIPCHK(hipMemsetAsync(h->d_band.p, 0, (size_t)ladder * per * sizeof(double), h->stream));
    } else if (P > LH_PMAX && h->opt.linear_solver == LH_SOLVER_LDLT) {   // k_ctrl_g's system, stride ceil32(6P); zeroed once
        const size_t ng = (size_t)((6 * P + 31) & ~31);
        h->lad_stride = ng * ng;   // one gA per ladder rung
        const bool fresh = h->d_gA.n < (size_t)ladder * ng * ng;
        HIPCHK(h->d_gA.ensure((size_t)ladder * ng * ng));
        if (fresh) HIPCHK(hipMemsetAsync(h->d_gA.p, 0, h->d_gA.n * sizeof(double), h->stream));
        // k_dense's dense symmetric S, double-buffered with the committed state
        const bool fresh_s = h->d_gS.n < 2 * ng * ng;
        HIPCHK(h->d_gS.ensure(2 * ng * ng));
        if (fresh_s) HIPCHK(hipMemsetAsync(h->d_gS.p, 0, h->d_gS.n * sizeof(double), h->stream));
    }

    // ---- k_ctrl's work units: the envelope of S in natural pose order ----
    if (P <= LH_PMAX) {
        int32_t fcb[8];
        for (int I = 0; I < 8; ++I) fcb[I] = 0;
        const int n = 6 * P, NE = (n + 15) & ~15;
        for (int I = 0; I < NE / 16; ++I) {
            int f = 1 << 20;
            for (int r = 16 * I; r < 16 * I + 16; ++r) f = std::min(f, r < n ? 6 * pf[r / 6] : r);
            fcb[I] = f >> 3;
        }
        // the two-chain schedule (opt-in, LH_ND=1): fewer steps where the window splits into decoupled
        // parts, but the separator's fill makes the early steps heavier; on C3 it measured slower than
        // the one-chain schedule
        h->nd.nsteps = 0;
        const char* nd_env = getenv("LH_ND");
        if (h->opt.linear_solver == LH_SOLVER_LDLT && nd_env && nd_env[0] == '1') lh_ctrl_nd_plan(P, pf.data(), h->nd);
        if (h->nd.nsteps > 0) {
            std::memcpy(h->s_units.p, h->nd.units, sizeof(h->nd.units));
        } else {
            const int order[15] = LH_ORDER_CTRL;
            lh_ctrl_units(6 * P, fcb, order, 15, LH_NSTEP, h->s_units.p);
        }
    } else {
        h->nd.nsteps = 0;
    }

    if (h->band) {
        std::memcpy(h->s_bunits.p, bunits.data(), bunits.size() * sizeof(uint16_t));
        int32_t* bb = h->s_bblk.p;
        for (size_t i = 0; i < (size_t)P * 64; ++i) bb[i] = -1;
        for (int b = 0; b < pl.npairs; ++b) {
            const int p = pl.pair_list[2 * b], q = pl.pair_list[2 * b + 1];
            if (q - p < 64) bb[p * 64 + (q - p)] = b;
        }
    }

    // ---- params ----
    lh_params& prm = h->prm;
    prm.P = P;
    prm.npairs = pl.npairs;
    prm.n = 6 * P;
    prm.ncam = ncam;
    prm.max_iters = h->opt.max_iters;
    prm.max_trials = h->opt.max_trials;
    prm.strategy = h->opt.strategy;
    prm.guard = h->opt.degenerate_guard;
    prm.gate_mode = h->opt.gate_mode;
    prm.precision = h->opt.precision;
    prm.lambda_given = h->opt.lambda_init >= 0.0;
    prm.ext_identity = ext_identity;
    prm.ext_rot_identity = ext_rot_identity;
    prm.huber_delta = h->opt.huber_delta;
    prm.stop_dchi2 = h->opt.stop_dchi2;
    prm.tau = h->opt.tau;
    prm.lambda_cap = h->opt.lambda_cap;
    prm.lambda_init = h->opt.lambda_init;
    prm.solver = h->opt.linear_solver;
    prm.pcg_tol = h->opt.pcg_tol;
    prm.pcg_max_it = h->opt.pcg_max_iters;
    prm.no_evo = getenv("LH_NO_EVO") != nullptr;
    prm.eval_first = getenv("LH_NO_EVAL_FIRST") == nullptr;
    prm.dec_in_reduce = dec1 ? 1 : 0;
    prm.batch = batch;
    prm.n_chunks = (int32_t)pl.n_chunks;
    prm.commit_in_reduce = h->band ? 1 : 0;
    // every controller builds the ladder: with k_reduce's decision (one rank, k_ctrl and k_ctrl_b) its rungs read it
    // from lh_ctrl; a controller that decides itself (the initial linearisation, sharded solves, k_ctrl_g, k_ctrl_p)
    // publishes its workgroup 0's decision to its rungs (ladder_publish / ladder_wait)
    prm.ladder = ladder;
    prm.lad_stride = (int32_t)h->lad_stride;
    // every factor builds the ladder (LH_LADDER_LAZY=1: only a factor after a rejection; the live configuration
    // measured 7 582 against 7 251 it/s, the headline window unchanged, profiles/r06c_*)
    prm.ladder_eager = getenv("LH_LADDER_LAZY") ? 0 : 1;
    prm.band_narrow = h->band_narrow ? 1 : 0;
    prm.band_lu = h->band_lu ? 1 : 0;
    // k_reduce writes the band straight into k_ctrl_b's loader order (one rank; LH_NO_BIMG=1: the packed
    // blocks and the loaders' block-index round trip, an A/B switch)
    prm.bimg = (h->band && prm.dec_in_reduce && !getenv("LH_NO_BIMG")) ? 1 : 0;
    if (prm.bimg) {   // entries no pair block writes stay zero: cleared per window
        const size_t nbi = 2 * (size_t)((6 * P + 15) >> 4) * LH_BIMG_TR;
        HIPCHK(h->d_img.ensure(nbi));
        HIPCHK(hipMemsetAsync(h->d_img.p, 0, nbi * sizeof(double), h->stream));
    }
    // k_reduce hands k_ctrl the system in its LDS layout (one rank, P <= LH_PMAX, the one-chain LDL^T;
    // LH_NO_IMG=1: the packed system and k_ctrl's scatter, an A/B switch)
    prm.img = (prm.dec_in_reduce && P <= LH_PMAX && h->opt.linear_solver == LH_SOLVER_LDLT && h->nd.nsteps == 0 &&
               !getenv("LH_NO_IMG")) ? 1 : 0;
    if (prm.img) {
        HIPCHK(h->d_img.ensure(2 * (size_t)LH_IMG_SZ));
        HIPCHK(lh_launch_img_init(h->stream, h->d_img.p, 6 * P));
    }
    prm.nd_steps = h->nd.nsteps;
    prm.nd_a = h->nd.a;
    prm.nd_s = h->nd.s;
    prm.nd_long_first = h->nd.long_first;
    for (int i = 0; i < 4; ++i) prm.K[i] = w->K[i];
    const double t1 = now_ms();

    // ---- the remaining copies ----
    hipStream_t s = h->stream;
    auto up = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
        if (!bytes) return hipSuccess;
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s);
    };
    HIPCHK(up(h->d_arena.p, h->s_arena.p, h->arena_bytes));   // every per-window table in one copy
    HIPCHK(hipEventRecord(h->ev_staging, s));
    h->staging_pending = true;
    if (sync) {
        HIPCHK(spin_wait(h->ev_staging));
        h->staging_pending = false;
    }
    h->last_prep_ms = t1 - t0;
    h->last_upload_ms = now_ms() - t0;
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

// One k_lin launch per tile count present.  In a trial, block 0 of the first launch (of a T = 1 launch
// with no chunks when the window has none) stores the trial's candidate poses and pose tables.
int launch_lin(lh_handle* h, int trial) {
    hipStream_t s = h->stream;
    // block 0 of the first launch: a trial's candidate poses and tables, or (the initial linearisation) the
    // restart of the solve from the uploaded window
    int writer = 1;
    const int P = h->P;
    const lh_reset_args rst{h->d_lm_perm.p, h->d_lm_in.p, h->d_qt_init.p, h->d_ptab_init.p, 24 * P,
                            (int)(2 * (size_t)P * h->ncam * LH_PT), 6 * std::max(P, 1)};
    for (int T = 1; T <= LH_TMAX; ++T) {
        const int c0 = h->plan.tgroup_begin[T], c1 = h->plan.tgroup_begin[T + 1];
        const bool last = T == LH_TMAX;
        if (c1 == c0 && !(writer && last)) continue;
        HIPCHK(lh_launch_lin(T, trial, c1 - c0, c0, s, h->d_chunks.p, h->d_sbs.p, h->d_uv.p, h->d_meta.p, h->d_rec.p,
                             h->d_ptab.p, h->d_ext.p, h->d_ctrl.p, h->d_dxp.p, h->d_rho.p, h->d_rows.p,
                             h->d_csc.p, h->d_items.p, h->d_wflag.p, (long)h->n_slots, h->prm, h->n_rec,
                             h->d_fixed.p, h->d_qt.p, writer, rst));
        writer = 0;
        DBGSYNC("k_lin");
    }
    return LH_OK;
}

// host-transport exchange: the reduced system (and at the initial linearisation max|diag H_ll|)
// through the caller's all-reduce, synchronously
int host_exchange(lh_handle* h, int mode) {
    hipStream_t s = h->stream;
    const size_t n = (size_t)h->LY.total;
    HIPCHK(hipMemcpyAsync(h->s_rs.p, h->d_rs_stage.p, n * sizeof(double), hipMemcpyDeviceToHost, s));
    if (mode == 0) HIPCHK(hipMemcpyAsync(h->s_rs.p + n, h->d_maxd.p, sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (mode == 0 && h->opt.allreduce(h->opt.allreduce_user, h->s_rs.p + n, 1, 1) != 0) return LH_E_RCCL;
    if (h->opt.allreduce(h->opt.allreduce_user, h->s_rs.p, (int64_t)n, 0) != 0) return LH_E_RCCL;
    ++h->n_coll;
    HIPCHK(hipMemcpyAsync(h->d_rs_stage.p, h->s_rs.p, n * sizeof(double), hipMemcpyHostToDevice, s));
    if (mode == 0) HIPCHK(hipMemcpyAsync(h->d_maxd.p, h->s_rs.p + n, sizeof(double), hipMemcpyHostToDevice, s));
    return LH_OK;
}

lh_band_args band_args(lh_handle* h) {
    if (!h->band) return lh_band_args{nullptr, nullptr, nullptr, nullptr};
    const size_t NE = (size_t)((6 * h->P + 15) & ~15);
    return lh_band_args{h->d_bblk.p, h->d_bunits.p, h->d_band.p, h->d_band.p + NE * 128};
}

// P2P: the exchange of chain `seq` (lh_launch_p2p; tags carry the solve count, so no stale tag ever matches)
hipError_t p2p_exchange(lh_handle* h, int mode, int seq) {
    const unsigned long long tag = ((unsigned long long)h->solve_gen << 32) | (unsigned long long)(seq + 1);
    ++h->n_coll;
    return lh_launch_p2p(h->stream, h->d_rs_stage.p, h->d_maxd.p, h->LY.total, h->peers, h->opt.rank, h->opt.world_size,
                         seq & 1, tag, h->xchg_slot, mode, h->d_xerr);
}

// One LM trial (mode 1) or the initial linearisation (mode 0).  *stopped is set (host transport
// only) when the device had already stopped: no exchange and no k_ctrl were issued.
int enqueue_trial(lh_handle* h, int mode, bool* stopped) {
    hipStream_t s = h->stream;
    h->cur_trial = (mode == 0) ? 0 : h->cur_trial + 1;
    {
        Prof pr(h, mode == 0 ? KC_INIT : KC_LIN);
        int st = launch_lin(h, mode);
        if (st != LH_OK) return st;
    }
    {
        Prof pr(h, KC_REDUCE);
        HIPCHK(lh_launch_reduce(s, h->d_rows.p, h->d_csc.p, h->d_red.p, h->n_red, h->d_ctrl.p,
                                h->d_rs_stage.p, h->d_rs_commit.p, h->d_maxd.p, h->prm, h->plan.n_chunks, mode, h->d_done,
                                h->cur_trial, h->d_img.p));
        DBGSYNC("k_reduce");
    }
    if (h->comm) {
        Prof pr(h, KC_ALLREDUCE);
        if (mode == 0) NCCLCHK(ncclAllReduce(h->d_maxd.p, h->d_maxd.p, 1, ncclFloat64, ncclMax, h->comm, s));
        NCCLCHK(ncclAllReduce(h->d_rs_stage.p, h->d_rs_stage.p, (size_t)h->LY.total, ncclFloat64, ncclSum, h->comm, s));
        ++h->n_coll;
    } else if (h->p2p) {
        Prof pr(h, KC_ALLREDUCE);
        HIPCHK(p2p_exchange(h, mode, h->cur_trial));
    } else if (h->host_comm) {
        HIPCHK(hipStreamSynchronize(s));
        if (mode != 0 && h->h_done[0]) {   // device-determined, identical on every rank
            *stopped = true;
            return LH_OK;
        }
        int st = host_exchange(h, mode);
        if (st != LH_OK) return st;
    }
    {
        Prof pr(h, KC_CTRL);
        if (h->P > LH_PMAX && h->prm.solver == LH_SOLVER_LDLT && !h->band)
            HIPCHK(lh_launch_dense(s, h->d_rs_stage.p, h->d_pair_pq.p, h->d_ctrl.p, h->d_gS.p, h->P));
        HIPCHK(lh_launch_ctrl(s, h->d_ctrl.p, h->d_rs_commit.p, h->d_rs_stage.p, h->d_maxd.p, h->d_rsmap.p, h->d_pair_pq.p,
                              h->d_dxp.p, h->prm, mode, h->d_done, h->cur_trial, h->d_gA.p, h->d_gS.p, h->d_brow_ptr.p,
                              h->d_brow_ent.p, h->d_units.p, band_args(h), h->d_img.p));
        DBGSYNC("k_ctrl");
    }
    return LH_OK;
}

// Results into the caller's buffers: device -> pinned staging in one stream (poses, landmark
// positions gathered into window order, per-edge rho0), then the staging is copied out on the
// planner's threads (a pageable device-to-host copy runs at a fraction of the link).
// the ABI-5 outlier flags were asked for (lh_result.is_outlier; read only at ABI 5)
bool wants_outliers(const lh_handle* h, const lh_result* out) {
    return out && h->opt.abi_version >= 5 && out->is_outlier != nullptr;
}

int download(lh_handle* h, lh_result* out, int cur) {
    hipStream_t s = h->stream;
    const int P = h->P;
    const double t0 = now_ms();
    const size_t np = out->pose_Tcw ? 12 * (size_t)P : 0;
    const size_t nl = (out->lm_xyz && h->L) ? 3 * (size_t)h->L : 0;
    const size_t ne = (out->edge_robust_chi2 && h->O) ? (size_t)h->O : 0;
    const bool fl = wants_outliers(h, out);
    const size_t o_res = ((size_t)h->O + 15) & ~(size_t)15;   // the scalars behind the flags: one copy
    if (fl) {   // Backend::Optimize's outlier pass on the device (backend_lego.cpp:163-194): flags + 3 scalars
        HIPCHK(h->d_ocnt.ensure(5 * 256));
        HIPCHK(h->d_oflag.ensure(o_res + 3 * sizeof(double)));
        HIPCHK(h->s_oflag.ensure(o_res + 3 * sizeof(double)));
        if (h->comm || h->host_comm) {
            // a sharded window: the reference counts the whole window's edges, so each rank counts its own, the
            // five counts and the edge counts are summed over the ranks (one 6-double exchange: every rank of the
            // handle asks for the flags alike, as it solves alike), and each rank flags its edges at the
            // threshold the totals give
            HIPCHK(h->d_otot.ensure(6));
            HIPCHK(lh_launch_outlier_counts(s, h->d_rho.p + h->rho_off, h->d_obs_perm.p, (long)h->n_slots, (long)h->O,
                                            out->outlier_chi2_th, h->d_ocnt.p, h->d_otot.p));
            if (h->comm) {
                NCCLCHK(ncclAllReduce(h->d_otot.p, h->d_otot.p, 6, ncclFloat64, ncclSum, h->comm, s));
            } else {
                double t6[6];
                HIPCHK(hipMemcpyAsync(t6, h->d_otot.p, sizeof(t6), hipMemcpyDeviceToHost, s));
                HIPCHK(hipStreamSynchronize(s));
                if (h->opt.allreduce(h->opt.allreduce_user, t6, 6, 0) != 0) return LH_E_RCCL;
                HIPCHK(hipMemcpyAsync(h->d_otot.p, t6, sizeof(t6), hipMemcpyHostToDevice, s));
                HIPCHK(hipStreamSynchronize(s));   // (t6 is on this stack frame)
            }
            HIPCHK(lh_launch_outlier_flags(s, h->d_rho.p + h->rho_off, h->d_obs_perm.p, (long)h->n_slots, (long)h->O,
                                           out->outlier_chi2_th, h->d_otot.p, h->d_oflag.p));
        } else {
            HIPCHK(lh_launch_outliers(s, h->d_rho.p + h->rho_off, h->d_obs_perm.p, (long)h->n_slots, (long)h->O, out->outlier_chi2_th,
                                      h->d_ocnt.p, h->d_oflag.p));
        }
        HIPCHK(hipMemcpyAsync(h->s_oflag.p, h->d_oflag.p, o_res + 3 * sizeof(double), hipMemcpyDeviceToHost, s));
    }
    if (np + nl + ne == 0 && !fl) {
        out->time_download_ms = 0.0;
        return LH_OK;
    }
    if (np + nl + ne == 0) {
        HIPCHK(hipStreamSynchronize(s));
        const uint8_t* sf = h->s_oflag.p;
        double r3[3];
        std::memcpy(r3, sf + o_res, sizeof(r3));
        out->outlier_th = r3[0];
        out->n_inlier = (int64_t)r3[1];
        out->n_outlier = (int64_t)r3[2];
        const ByteSeg seg_f = {out->is_outlier, sf, (size_t)h->O};
        par_copy(h, &seg_f, 1);
        out->time_download_ms = now_ms() - t0;
        return LH_OK;
    }
    HIPCHK(h->s_out.ensure(np + nl + ne));
    double* st = h->s_out.p;
    if (np)   // estimate_ of every VertexPose (backend_lego.cpp:198-213)
        HIPCHK(hipMemcpyAsync(st, h->d_qt.p + 12 * (size_t)cur * P, np * sizeof(double), hipMemcpyDeviceToHost, s));
    if (nl || ne) {
        // landmarks without an edge are not vertices (backend_lego.cpp:126): they keep their input
        if (nl) HIPCHK(hipMemcpyAsync(h->d_out_xyz.p, h->d_lm_in.p, nl * sizeof(double), hipMemcpyDeviceToDevice, s));
        HIPCHK(lh_launch_gather(s, h->d_ctrl.p, h->d_rec.p, h->d_lm_perm.p, nl ? h->n_rec : 0, h->d_rho.p + h->rho_off,
                                h->d_obs_perm.p, ne ? (long)h->n_slots : 0L, h->d_out_xyz.p, h->d_out_rho.p));
        if (nl) HIPCHK(hipMemcpyAsync(st + np, h->d_out_xyz.p, nl * sizeof(double), hipMemcpyDeviceToHost, s));
    }
    // poses and landmarks are copied out of the staging while the per-edge chi2 is still in flight
    hipEvent_t e_first = next_event(h);
    if (!e_first) return LH_E_HIP;
    HIPCHK(hipEventRecord(e_first, s));
    if (ne) HIPCHK(hipMemcpyAsync(st + np + nl, h->d_out_rho.p, ne * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(spin_wait(e_first));
    const ByteSeg seg[2] = {{out->pose_Tcw, st, np * sizeof(double)}, {out->lm_xyz, st + np, nl * sizeof(double)}};
    par_copy(h, seg, 2);
    HIPCHK(hipStreamSynchronize(s));
    const ByteSeg seg_e[2] = {{out->edge_robust_chi2, st + np + nl, ne * sizeof(double)},
                              {fl ? out->is_outlier : nullptr, fl ? h->s_oflag.p : nullptr, fl ? (size_t)h->O : 0}};
    par_copy(h, seg_e, 2);
    if (fl) {
        double r3[3];
        std::memcpy(r3, h->s_oflag.p + o_res, sizeof(r3));
        out->outlier_th = r3[0];
        out->n_inlier = (int64_t)r3[1];
        out->n_outlier = (int64_t)r3[2];
    }
    out->time_download_ms = now_ms() - t0;
    return LH_OK;
}

int solve_resident_impl(lh_handle* h, lh_result* out) {
    if (!h->uploaded) return LH_E_STATE;
    hipStream_t s = h->stream;
    hipEvent_t e0 = next_event(h), e1 = next_event(h);
    if (!e0 || !e1) return LH_E_HIP;
    volatile int* hd = h->h_done;   // [0] done, [1] progress word (ctrl_lm_step)
    hd[0] = 0;
    hd[1] = -1;
    // No arrays wanted (and no collectives, profiling or printout): the summary comes with done in the
    // mapped words, and the solve returns when the host sees it; later work on this handle is stream-
    // ordered behind the solve's kernels (lh_destroy synchronises)
    const bool fast = out && !out->pose_Tcw && !out->lm_xyz && !out->edge_robust_chi2 && !wants_outliers(h, out) &&
                      !h->comm && !h->host_comm && !h->p2p && !h->opt.profile && !h->opt.verbose;
    const double t_start = now_ms();
    h->n_coll = 0;
    if (h->p2p) {
        ++h->solve_gen;   // every rank solves the same number of times
        if (*h->h_xerr) return LH_E_RCCL;   // an earlier exchange failed: the peers are not in step
    }
    if (!fast) HIPCHK(hipEventRecord(e0, s));   // (the array-free solve times itself on the host clock)
    // (the restart -- controller, poses, tables, step -- is the initial linearisation's block 0, launch_lin)
    bool stopped = false;
    int st = enqueue_trial(h, 0, &stopped);
    if (st != LH_OK) return st;
    // every trial, plus one re-linearisation chain per iteration at most (an evaluate-only acceptance, ctrl.relin)
    const int max_total = (h->opt.max_iters > 0) ? h->opt.max_iters * (std::max(1, h->opt.max_trials) + (h->prm.eval_first ? 1 : 0)) : 0;
    const int depth = h->host_comm ? 1 : (h->opt.trials_per_sync > 0 ? std::min(h->opt.trials_per_sync, 32) : 2);
    int enq = 0;
    if (h->host_comm) {
        // synchronous: each trial's exchange waits for the previous k_ctrl, whose stop flag every
        // rank reads at the same point
        while (enq < max_total && !stopped) {
            if ((st = enqueue_trial(h, 1, &stopped)) != LH_OK) return st;
            if (!stopped) ++enq;
        }
    } else {
        // k_ctrl writes each live trial it has decided into the mapped progress word; the host
        // keeps `depth` trials enqueued past it (one when the next completed iteration reaches
        // max_iters) until the device raises done.  hipStreamQuery at most every 50 ms turns a
        // device fault into an error return (each query delays the next launch by ~6 us).
        unsigned spin = 0;
        static const bool query_often = getenv("LH_QUERY_OFTEN") != nullptr;   // diagnostic A/B switch (timing only)
        double t_query = now_ms();
        while (!hd[0] && enq < max_total) {
            const int pw = hd[1];   // 2 * (last live trial) + near, or -1 before the first
            const int last = pw < 0 ? -1 : (pw >> 1);
            if (enq - last < ((pw >= 0 && (pw & 1)) ? 1 : depth)) {
                if ((st = enqueue_trial(h, 1, &stopped)) != LH_OK) return st;
                ++enq;
                continue;
            }
            if ((++spin & 4095) == 0 && (query_often || now_ms() - t_query > 50.0)) {
                const hipError_t q = hipStreamQuery(s);
                if (q != hipSuccess && q != hipErrorNotReady) return LH_E_HIP;
                if (h->p2p && *h->h_xerr) {   // a peer's tag did not arrive (k_p2p_sum gave up)
                    (void)hipStreamSynchronize(s);
                    return LH_E_RCCL;
                }
                t_query = now_ms();
            }
            __builtin_ia32_pause();
        }
    }
    if (fast) {
        // every trial is enqueued: the device raises done on the last one (max_iters x max_trials trials
        // reach max_iters); a fault, or an idle stream without done, ends the wait with an error
        double t_query = now_ms();
        unsigned spin = 0;
        while (!hd[0]) {
            if ((++spin & 4095) == 0 && now_ms() - t_query > 50.0) {
                const hipError_t q = hipStreamQuery(s);
                if (q == hipSuccess && !hd[0]) return LH_E_STATE;
                if (q != hipSuccess && q != hipErrorNotReady) return LH_E_HIP;
                t_query = now_ms();
            }
            __builtin_ia32_pause();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        const volatile lh_host_words* hw = reinterpret_cast<const volatile lh_host_words*>(h->h_done);
        out->iterations = hw->iter;
        out->trials = hw->trials;
        out->accepted = hw->accepted;
        out->chi2_initial = hw->chi2_initial;
        out->chi2_final = hw->chi;
        out->lambda_final = hw->lambda;
        out->time_ms = now_ms() - t_start;   // host clock: enqueue of the first kernel to done seen
        out->pcg_iterations = hw->pcg_iters;
        out->degenerate = hw->nonpd;
        out->trace_len = std::min((int)hw->trace_len, std::min(out->trace_cap, LH_TRACE));
        for (int i = 0; i < out->trace_len; ++i) {
            if (out->trace_chi2) out->trace_chi2[i] = hw->trace_chi[i];
            if (out->trace_lambda) out->trace_lambda[i] = hw->trace_lambda[i];
        }
        out->time_prep_ms = h->last_prep_ms;
        out->time_upload_ms = h->last_upload_ms;
        out->time_download_ms = 0.0;
        h->event_next = 0;
        h->last_chains = -1;   // (not in the host words)
        h->last_lskips = -1;
        return LH_OK;
    }
    HIPCHK(hipEventRecord(e1, s));
    HIPCHK(hipMemcpyAsync(h->h_ctrl, h->d_ctrl.p, sizeof(lh_ctrl), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const lh_ctrl& c = *h->h_ctrl;
    if (h->comm || h->p2p) {
        // Equal collective counts on every rank.  The progress word only advances on live chains,
        // so no rank enqueued more than (stop chain) + depth chains; the stop chain is decided by
        // identical all-reduced data, so every rank tops up to the same target.  The extra
        // all-reduces carry no data anyone reads (the device has stopped).
        const int target = std::min(c.seq_last + depth, max_total);
        if (enq > target) return LH_E_STATE;   // cannot happen: the bound above
        for (; enq < target; ++enq) {
            if (h->p2p) {
                HIPCHK(p2p_exchange(h, 1, ++h->cur_trial));   // the chain numbers continue as the trials' did
            } else {
                NCCLCHK(ncclAllReduce(h->d_rs_stage.p, h->d_rs_stage.p, (size_t)h->LY.total, ncclFloat64, ncclSum, h->comm, s));
                ++h->n_coll;
            }
        }
        HIPCHK(hipStreamSynchronize(s));
        if (h->p2p && *h->h_xerr) return LH_E_RCCL;
    }
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    const int cur = c.cur;
    h->rho_off = (size_t)c.rho_sel * h->n_slots;
    h->last_batches = c.nbatches;
    h->last_retrials[0] = c.nretrials[0];
    h->last_retrials[1] = c.nretrials[1];
    h->last_chains = c.seq_last;
    h->last_lskips = c.lskips;

    if (out) {
        out->iterations = c.iter;
        out->trials = c.trials;
        out->accepted = c.accepted;
        out->chi2_initial = c.chi2_initial;
        out->chi2_final = c.chi;
        out->lambda_final = c.lambda;
        out->time_ms = ms;
        out->pcg_iterations = c.pcg_iters;
        out->degenerate = c.nonpd;
        out->trace_len = std::min(c.trace_len, std::min(out->trace_cap, LH_TRACE));
        for (int i = 0; i < out->trace_len; ++i) {
            if (out->trace_chi2) out->trace_chi2[i] = c.trace_chi[i];
            if (out->trace_lambda) out->trace_lambda[i] = c.trace_lambda[i];
        }
        out->time_prep_ms = h->last_prep_ms;
        out->time_upload_ms = h->last_upload_ms;
        out->time_download_ms = 0.0;
        st = download(h, out, cur);
        if (st != LH_OK) return st;
    }
    if (h->opt.verbose) {
        printf("==========LEGO OPTIMIZER (MI355X)==========\n");
        for (int i = 0; i < std::min(c.trace_len, LH_TRACE); ++i)
            printf("Iteration = %d,\tChi = %g,\tLambda = %g\n", i, c.trace_chi[i], c.trace_lambda[i]);
        printf("\nInfo: \nTimeCost(SolveProblem) = %g ms\n", (double)ms);
    }
    if (h->opt.profile) collect_profile(h, c.seq_last);
    else h->event_next = 0;
    return LH_OK;
}

// Every rank must run the same controller with the same options: the LM decisions are taken on
// identical all-reduced sums, and the number of collectives a solve issues is a function of the stop
// trial, the enqueue depth and max_iters x max_trials (solve_resident_impl).  Ranks whose options
// differ would issue different collective counts and hang, so lh_create compares them once: each
// rank contributes (v, -v) per option to a MAX all-reduce, and any rank whose v differs from the
// maximum or minimum sees a mismatch (every rank returns LH_E_BADARG).
// MAX over the ranks of buf[0..n), in place (host transport or RCCL); a no-op on one rank
int rank_max(lh_handle* h, double* buf, int n) {
    if (h->host_comm || h->p2p) {
        if (h->opt.allreduce(h->opt.allreduce_user, buf, n, 1) != 0) return LH_E_RCCL;
    } else if (h->comm) {
        DevBuf<double> d;
        auto run = [&]() -> int {
            HIPCHK(d.ensure(n));
            HIPCHK(hipMemcpyAsync(d.p, buf, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
            NCCLCHK(ncclAllReduce(d.p, d.p, n, ncclFloat64, ncclMax, h->comm, h->stream));
            HIPCHK(hipMemcpyAsync(buf, d.p, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
            HIPCHK(hipStreamSynchronize(h->stream));
            return LH_OK;
        };
        const int st = run();
        d.release();
        return st;
    }
    return LH_OK;
}

// P2P: this rank's exchange buffer (2 parities x world slots of the packed reduced system + max|diag H_ll|, then
// the arrival tags), exported over IPC, and every peer's opened here.  Collective: every rank calls it at the same
// upload (the buffer size follows from the reduced system's layout, identical on every rank); its handles travel
// through the caller's all-reduce (a sum of byte values, exact), and a MAX all-reduce of the status ends it, so a
// rank that cannot map a peer takes every rank's upload down with it.
int p2p_setup(lh_handle* h) {
    const int world = h->opt.world_size, rank = h->opt.rank;
    const long slot = (h->LY.total + 1 + 63) & ~63L;
    const size_t need = (size_t)2 * world * slot + 2 * (size_t)world;   // (a tag is one 8-byte word)
    if (h->d_xchg.n >= need && h->xchg_slot == slot) return LH_OK;
    int st = LH_OK;
    for (int r = 0; r < world; ++r)
        if (r != rank && h->peers.p[r]) (void)hipIpcCloseMemHandle(h->peers.p[r]);
    h->peers = lh_peers{};
    h->d_xchg.release();
    hipIpcMemHandle_t mine{};
    if (h->d_xchg.ensure(need) != hipSuccess ||
        hipMemsetAsync(h->d_xchg.p, 0, need * sizeof(double), h->stream) != hipSuccess ||
        hipStreamSynchronize(h->stream) != hipSuccess || hipIpcGetMemHandle(&mine, h->d_xchg.p) != hipSuccess)
        st = LH_E_HIP;
    static_assert(sizeof(hipIpcMemHandle_t) <= 64, "an IPC handle in 64 byte values");
    std::vector<double> hb((size_t)world * 64, 0.0);
    const uint8_t* mb = reinterpret_cast<const uint8_t*>(&mine);
    for (size_t i = 0; i < sizeof(mine); ++i) hb[(size_t)rank * 64 + i] = (double)mb[i];
    if (h->opt.allreduce(h->opt.allreduce_user, hb.data(), (int64_t)hb.size(), 0) != 0) return LH_E_RCCL;
    h->peers.p[rank] = h->d_xchg.p;
    for (int r = 0; r < world && st == LH_OK; ++r) {
        if (r == rank) continue;
        hipIpcMemHandle_t ph{};
        uint8_t* pb = reinterpret_cast<uint8_t*>(&ph);
        for (size_t i = 0; i < sizeof(ph); ++i) pb[i] = (uint8_t)hb[(size_t)r * 64 + i];
        void* p = nullptr;
        if (hipIpcOpenMemHandle(&p, ph, hipIpcMemLazyEnablePeerAccess) != hipSuccess || !p) {
            if (getenv("LH_DEBUG_P2P")) fprintf(stderr, "lego_ba: rank %d cannot map rank %d's exchange buffer\n", rank, r);
            st = LH_E_UNSUPPORTED;
        } else {
            h->peers.p[r] = static_cast<double*>(p);
        }
    }
    double fs = (double)st;
    const int st_r = rank_max(h, &fs, 1);
    if (st_r != LH_OK) return st_r;
    if (fs > 0.0) return (int)fs;
    h->xchg_slot = slot;
    return LH_OK;
}

int check_rank_options(lh_handle* h) {
    const lh_options& o = h->opt;
    const int depth = h->host_comm ? 1 : (o.trials_per_sync > 0 ? std::min(o.trials_per_sync, 32) : 2);
    const double v[] = {(double)o.max_iters, (double)o.max_trials, (double)o.strategy, o.huber_delta, o.stop_dchi2,
                        o.tau, o.lambda_cap, o.lambda_init, (double)o.linear_solver, (double)o.world_size,
                        (double)o.degenerate_guard, (double)depth, (double)o.pcg_max_iters, o.pcg_tol,
                        (double)o.gate_mode, (double)o.chunk_landmarks > 0 ? 1.0 : 0.0, (double)o.comm_mode,
                        (double)o.precision};
    constexpr int n = (int)(sizeof(v) / sizeof(v[0]));
    double buf[2 * n];
    for (int i = 0; i < n; ++i) { buf[i] = v[i]; buf[n + i] = -v[i]; }
    if (!h->host_comm && !h->comm && !h->p2p) return LH_OK;
    const int st = rank_max(h, buf, 2 * n);
    if (st != LH_OK) return st;
    for (int i = 0; i < n; ++i)
        if (!(buf[i] == -buf[n + i])) return LH_E_BADARG;   // max != min somewhere (NaN options fail too)
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
        case LH_E_RCCL: return "RCCL / exchange error";
        case LH_E_UNSUPPORTED: return "window outside the supported envelope";
        case LH_E_STATE: return "call out of order";
        default: return "unknown status";
    }
}

const char* lh_kernel_name(int kc) { return (kc >= 0 && kc < KC_N) ? kKernelNames[kc] : ""; }

// (the exported symbol, not the header's macro: binaries built against the ABI-4 header call it by this name)
#undef lh_default_options
void lh_default_options(lh_options* o) { lh_default_options_v(o, 4); }

void lh_default_options_v(lh_options* o, int abi) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->abi_version = abi;
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
    o->gate_mode = 0;
    o->chunk_landmarks = 0;
    o->comm_mode = LH_COMM_RCCL;
    o->host_threads = 0;
    o->allreduce = nullptr;
    o->allreduce_user = nullptr;
    o->precision = LH_PREC_FP64;
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
    if (opt->abi_version != LH_ABI_VERSION && opt->abi_version != 4) return LH_E_BADARG;
    if (opt->max_iters < 0 || opt->max_trials < 0 || opt->world_size < 1 || opt->rank < 0 ||
        opt->rank >= opt->world_size || (opt->strategy != 0 && opt->strategy != 1))
        return LH_E_BADARG;
    if (opt->linear_solver != LH_SOLVER_LDLT && opt->linear_solver != LH_SOLVER_PCG) return LH_E_BADARG;
    if (opt->linear_solver == LH_SOLVER_PCG && !(opt->pcg_tol >= 0.0)) return LH_E_BADARG;
    if (opt->gate_mode != 0 && opt->gate_mode != 1) return LH_E_BADARG;
    if (opt->precision != LH_PREC_FP64 && opt->precision != LH_PREC_FP32_RESID) return LH_E_BADARG;
    if (opt->degenerate_guard != 0 && opt->degenerate_guard != 1) return LH_E_BADARG;
    if (opt->chunk_landmarks < 0 || opt->host_threads < 0) return LH_E_BADARG;
    if (opt->comm_mode != LH_COMM_RCCL && opt->comm_mode != LH_COMM_HOST && opt->comm_mode != LH_COMM_P2P)
        return LH_E_BADARG;
    if (opt->world_size > 1 && opt->comm_mode != LH_COMM_RCCL && !opt->allreduce) return LH_E_BADARG;
    if (opt->comm_mode == LH_COMM_P2P && opt->world_size > LH_P2P_MAX) return LH_E_UNSUPPORTED;
    lh_handle* h = new (std::nothrow) lh_handle();
    if (!h) return LH_E_HIP;
    h->opt = *opt;
    int dev = opt->device;
    if (dev < 0) {
        if (hipGetDevice(&dev) != hipSuccess) { delete h; return LH_E_HIP; }
    }
    if (hipSetDevice(dev) != hipSuccess) { delete h; return LH_E_HIP; }
    h->device = dev;
    int lds = 0;
    if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) == hipSuccess && lds > 0)
        h->lds_limit = lds;
    if (lh_prepare_lin(h->lds_limit) != hipSuccess) { delete h; return LH_E_HIP; }
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) { delete h; return LH_E_HIP; }
    if (hipHostMalloc((void**)&h->h_ctrl, sizeof(lh_ctrl), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&h->h_done, sizeof(lh_host_words), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&h->d_done, h->h_done, 0) != hipSuccess) {
        lh_destroy(h);
        return LH_E_HIP;
    }
    // the pool starts std::threads, which throw std::system_error when the process may not create
    // more (e.g. under a cgroup pids limit): no exception crosses the ABI
    try {
        h->pool = new lh::Pool(opt->host_threads > 0 ? std::min(opt->host_threads, 64) : auto_host_threads());
    } catch (...) {
        h->pool = nullptr;
    }
    if (!h->pool) { lh_destroy(h); return LH_E_HIP; }
    if (hipEventCreateWithFlags(&h->ev_staging, hipEventDisableTiming) != hipSuccess) {
        h->ev_staging = nullptr;
        lh_destroy(h);
        return LH_E_HIP;
    }
    h->host_comm = opt->world_size > 1 && opt->comm_mode == LH_COMM_HOST;
    h->p2p = opt->world_size > 1 && opt->comm_mode == LH_COMM_P2P;
    if (h->p2p) {
        if (hipHostMalloc((void**)&h->h_xerr, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void**)&h->d_xerr, h->h_xerr, 0) != hipSuccess) {
            lh_destroy(h);
            return LH_E_HIP;
        }
        *h->h_xerr = 0;
    }
    // LH_FORCE_RCCL=1 builds a one-rank communicator on a single GPU, so the data-path
    // collectives (and their stream ordering) run in single-GPU tests too
    const char* force = std::getenv("LH_FORCE_RCCL");
    const bool force_comm = opt->world_size == 1 && force && force[0] == '1';
    if ((opt->world_size > 1 && !h->host_comm && !h->p2p) || force_comm) {
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
    if (opt->world_size > 1) {
        const int st = check_rank_options(h);
        if (st != LH_OK) { lh_destroy(h); return st; }
    }
    *hp = h;
    return LH_OK;
}

void lh_destroy(lh_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->comm) ncclCommDestroy(h->comm);
    for (int r = 0; r < LH_P2P_MAX; ++r)
        if (h->peers.p[r] && h->peers.p[r] != h->d_xchg.p) (void)hipIpcCloseMemHandle(h->peers.p[r]);
    h->d_xchg.release();
    if (h->h_xerr) (void)hipHostFree(h->h_xerr);
    for (auto e : h->event_pool) (void)hipEventDestroy(e);
    delete h->pool;
    h->f_in.release(); h->f_out.release(); h->f_res.release(); h->s_fin.release(); h->s_fout.release();
    h->k_img[0].release(); h->k_img[1].release(); h->k_succ.release(); h->k_kp1.release(); h->k_kp2.release();
    h->d_chunks.release(); h->d_sbs.release(); h->d_meta.release(); h->d_obs_perm.release(); h->d_lm_perm.release();
    h->d_pair_ptr.release(); h->d_items.release(); h->d_pair_pq.release(); h->d_lm_in.release();
    h->d_uv.release(); h->d_rec.release(); h->d_ptab.release(); h->d_out_xyz.release(); h->d_out_rho.release();
    h->d_ptab_init.release(); h->d_qt.release(); h->d_qt_init.release(); h->d_ext.release(); h->d_rho.release();
    h->d_rows.release(); h->d_csc.release(); h->d_gA.release(); h->d_gS.release(); h->d_rs_stage.release(); h->d_rs_commit.release(); h->d_rsmap.release(); h->d_maxd.release(); h->d_band.release();
    h->d_dxp.release(); h->d_ctrl.release(); h->d_wflag.release(); h->d_img.release(); h->d_fixed.release();
    h->d_brow_ptr.release(); h->d_brow_ent.release(); h->d_arena.release(); h->s_arena.release();
    h->s_chunks.release(); h->s_sbs.release(); h->s_meta.release(); h->s_items.release(); h->s_pair_ptr.release();
    h->s_rsmap.release(); h->s_pair_pq.release(); h->s_obs_perm.release(); h->s_lm_perm.release(); h->s_uv.release();
    h->s_lm.release(); h->s_qt.release(); h->s_ptab.release(); h->s_ext.release(); h->s_rs.release();
    h->s_out.release();
    h->d_ocnt.release(); h->d_oflag.release(); h->s_oflag.release(); h->d_otot.release();
    if (h->ev_staging) (void)hipEventDestroy(h->ev_staging);
    if (h->h_ctrl) (void)hipHostFree(h->h_ctrl);
    if (h->h_done) (void)hipHostFree(h->h_done);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int lh_upload(lh_handle* h, const lh_window* in) {
    if (!h) return LH_E_BADARG;
    if (hipSetDevice(h->device) != hipSuccess) return LH_E_HIP;
    try {
        return upload_impl(h, in, true);
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
    if (!h) return LH_E_BADARG;
    if (hipSetDevice(h->device) != hipSuccess) return LH_E_HIP;
    int st;
    try {
        st = upload_impl(h, in, false);   // the copies stay queued ahead of the solve's kernels
    } catch (const std::bad_alloc&) {
        return LH_E_HIP;
    } catch (...) {
        return LH_E_BADARG;
    }
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
static int estimate_pose_impl(lh_handle* h, const lh_frames* in, lh_frames_result* out) {
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
    // arena layouts (16-byte aligned segments)
    auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
    const bool has_flag = in->is_outlier && O > 0;
    const size_t i_ptr = 0, i_pose = al(sizeof(int64_t) * (F + 1)), i_pts = i_pose + al(sizeof(double) * 12 * (size_t)F),
                 i_uv = i_pts + al(sizeof(double) * 3 * (size_t)O), i_flag = i_uv + al(sizeof(double) * 2 * (size_t)O),
                 i_end = i_flag + (has_flag ? al((size_t)O) : 0);
    const size_t o_pose = 0, o_rchi2 = al(sizeof(double) * 12 * (size_t)F), o_iters = o_rchi2 + al(sizeof(double) * (size_t)O),
                 o_inl = o_iters + al(sizeof(int32_t) * (size_t)F), o_flag = o_inl + al(sizeof(int32_t) * (size_t)F),
                 o_end = o_flag + al((size_t)O);
    HIPCHK(h->f_in.ensure(i_end));
    HIPCHK(h->f_out.ensure(o_end));
    HIPCHK(h->f_res.ensure(2 * (size_t)O));
    HIPCHK(h->s_fin.ensure(i_end));
    HIPCHK(h->s_fout.ensure(o_end));
    {
        uint8_t* st = h->s_fin.p;
        const ByteSeg seg[5] = {{st + i_ptr, in->obs_ptr, sizeof(int64_t) * (F + 1)},
                                {st + i_pose, in->pose_Tcw, sizeof(double) * 12 * (size_t)F},
                                {st + i_pts, in->pts_w, sizeof(double) * 3 * (size_t)O},
                                {st + i_uv, in->obs_uv, sizeof(double) * 2 * (size_t)O},
                                {st + i_flag, in->is_outlier, has_flag ? (size_t)O : 0}};
        par_copy(h, seg, 5);
    }
    HIPCHK(hipMemcpyAsync(h->f_in.p, h->s_fin.p, i_end, hipMemcpyHostToDevice, s));
    uint8_t* fi = h->f_in.p;
    uint8_t* fo = h->f_out.p;
    lh_params prm{};
    prm.max_iters = h->opt.max_iters;
    prm.max_trials = h->opt.max_trials;
    prm.strategy = h->opt.strategy;
    prm.lambda_given = h->opt.lambda_init >= 0.0;
    prm.gate_mode = h->opt.gate_mode;
    prm.precision = h->opt.precision;
    prm.huber_delta = h->opt.huber_delta;
    prm.stop_dchi2 = h->opt.stop_dchi2;
    prm.tau = h->opt.tau;
    prm.lambda_cap = h->opt.lambda_cap;
    prm.lambda_init = h->opt.lambda_init;
    for (int i = 0; i < 4; ++i) prm.K[i] = in->K[i];
    hipEvent_t e0 = next_event(h), e1 = next_event(h);
    if (!e0 || !e1) return LH_E_HIP;
    HIPCHK(hipEventRecord(e0, s));
    HIPCHK(lh_launch_frames(s, F, (const int64_t*)(fi + i_ptr), (const double*)(fi + i_pose),
                            (const double*)(fi + i_pts), (const double*)(fi + i_uv), has_flag ? fi + i_flag : nullptr,
                            prm, h->f_res.p, (double*)(fo + o_pose), fo + o_flag, (double*)(fo + o_rchi2),
                            (int32_t*)(fo + o_iters), (int32_t*)(fo + o_inl)));
    HIPCHK(hipEventRecord(e1, s));
    // one download of what the caller asked for: the pose block always, the rest up to the last wanted
    const size_t want = out->is_outlier && O > 0 ? o_end
                        : out->n_inliers         ? o_flag
                        : out->iterations        ? o_inl
                        : out->edge_chi2 && O > 0 ? o_iters
                                                 : o_rchi2;
    HIPCHK(hipMemcpyAsync(h->s_fout.p, fo, want, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    {
        const uint8_t* st = h->s_fout.p;
        const ByteSeg seg[5] = {{out->pose_Tcw, st + o_pose, sizeof(double) * 12 * (size_t)F},
                                {out->edge_chi2, st + o_rchi2, out->edge_chi2 ? sizeof(double) * (size_t)O : 0},
                                {out->iterations, st + o_iters, out->iterations ? sizeof(int32_t) * (size_t)F : 0},
                                {out->n_inliers, st + o_inl, out->n_inliers ? sizeof(int32_t) * (size_t)F : 0},
                                {out->is_outlier, st + o_flag, out->is_outlier ? (size_t)O : 0}};
        par_copy(h, seg, 5);
    }
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    out->time_ms = ms;
    h->event_next = 0;
    return LH_OK;
}

// LKOpticalFlow4Layer / LKOpticalFlow1Layer (algorithm.cpp:11-206): upload both images, build the
// pyramids (k_lk_pyr per level and image), track every keypoint (k_lk_track), download.
static int lk_track_impl(lh_handle* h, const lh_lk_input* in, lh_lk_result* out) {
    if (!h || !in || !out) return LH_E_BADARG;
    if (in->levels != 1 && in->levels != LH_LK_MAX_LEVELS) return LH_E_BADARG;
    if (in->cols < 1 || in->rows < 1 || in->step < in->cols || in->n_points < 0) return LH_E_BADARG;
    if (!in->img1 || !in->img2) return LH_E_BADARG;
    const int n = in->n_points;
    if (n > 0 && (!in->kp1 || !out->kp2 || !out->success)) return LH_E_BADARG;
    if (hipSetDevice(h->device) != hipSuccess) return LH_E_HIP;
    // level sizes: cv::Size(cols * 0.5, rows * 0.5) truncated (algorithm.cpp:146-153)
    int cols[LH_LK_MAX_LEVELS], rows[LH_LK_MAX_LEVELS];
    int64_t step[LH_LK_MAX_LEVELS], off[LH_LK_MAX_LEVELS];
    cols[0] = in->cols; rows[0] = in->rows; step[0] = in->step; off[0] = 0;
    int64_t total = (int64_t)in->rows * in->step;
    for (int l = 1; l < in->levels; ++l) {
        cols[l] = (int)(cols[l - 1] * 0.5);
        rows[l] = (int)(rows[l - 1] * 0.5);
        if (cols[l] < 1 || rows[l] < 1) return LH_E_BADARG;
        step[l] = cols[l];
        off[l] = total;
        total += (int64_t)cols[l] * rows[l];
    }
    hipStream_t s = h->stream;
    HIPCHK(h->k_img[0].ensure((size_t)total));
    HIPCHK(h->k_img[1].ensure((size_t)total));
    HIPCHK(h->k_kp1.ensure(2 * (size_t)std::max(n, 1)));
    HIPCHK(h->k_kp2.ensure(2 * (size_t)std::max(n, 1)));
    HIPCHK(h->k_succ.ensure((size_t)std::max(n, 1)));
    // the caller's last row guarantees only `cols` readable bytes (a cv::Mat ROI has step > cols):
    // copy (rows - 1) * step + cols bytes and zero the rest of that row, which no tap reads as image
    // data (GetPixelValue's out-of-buffer taps read 0, lh_lk.hip)
    const size_t img_bytes = (size_t)(in->rows - 1) * (size_t)in->step + (size_t)in->cols;
    const size_t tail = (size_t)in->rows * (size_t)in->step - img_bytes;
    for (int im = 0; im < 2; ++im) {
        HIPCHK(hipMemcpyAsync(h->k_img[im].p, im ? in->img2 : in->img1, img_bytes, hipMemcpyHostToDevice, s));
        if (tail) HIPCHK(hipMemsetAsync(h->k_img[im].p + img_bytes, 0, tail, s));
    }
    if (n > 0) {
        HIPCHK(hipMemcpyAsync(h->k_kp1.p, in->kp1, 2 * sizeof(float) * (size_t)n, hipMemcpyHostToDevice, s));
        // without an initial guess kp2 is scaled but never read (dx = dy = 0 at the top level)
        if (in->has_initial) HIPCHK(hipMemcpyAsync(h->k_kp2.p, out->kp2, 2 * sizeof(float) * (size_t)n, hipMemcpyHostToDevice, s));
        else HIPCHK(hipMemsetAsync(h->k_kp2.p, 0, 2 * sizeof(float) * (size_t)n, s));
    }
    lh_lk_levels L[2];
    for (int im = 0; im < 2; ++im)
        for (int l = 0; l < LH_LK_MAX_LEVELS; ++l) {
            const int ll = l < in->levels ? l : 0;
            L[im].data[l] = h->k_img[im].p + off[ll];
            L[im].cols[l] = cols[ll];
            L[im].rows[l] = rows[ll];
            L[im].step[l] = step[ll];
        }
    hipEvent_t e0 = next_event(h), e1 = next_event(h);
    if (!e0 || !e1) return LH_E_HIP;
    HIPCHK(hipEventRecord(e0, s));
    for (int l = 1; l < in->levels; ++l)
        for (int im = 0; im < 2; ++im)
            HIPCHK(lh_launch_lk_pyr(s, L[im].data[l - 1], cols[l - 1], rows[l - 1], step[l - 1],
                                    h->k_img[im].p + off[l], cols[l], rows[l]));
    HIPCHK(lh_launch_lk_track(s, &L[0], &L[1], in->levels, n, h->k_kp1.p, h->k_kp2.p, h->k_kp2.p, h->k_succ.p,
                              in->inverse ? 1 : 0, in->has_initial ? 1 : 0));
    HIPCHK(hipEventRecord(e1, s));
    if (n > 0) {
        HIPCHK(hipMemcpyAsync(out->kp2, h->k_kp2.p, 2 * sizeof(float) * (size_t)n, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(out->success, h->k_succ.p, (size_t)n, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    out->time_ms = ms;
    h->event_next = 0;
    return LH_OK;
}

// the staging copies build std::vectors (par_copy): no exception crosses the ABI
int lh_estimate_pose(lh_handle* h, const lh_frames* in, lh_frames_result* out) {
    try {
        return estimate_pose_impl(h, in, out);
    } catch (...) {
        return LH_E_HIP;
    }
}

int lh_lk_track(lh_handle* h, const lh_lk_input* in, lh_lk_result* out) {
    try {
        return lk_track_impl(h, in, out);
    } catch (...) {
        return LH_E_HIP;
    }
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
    // an array-free solve returns before its stream drains (solve_resident_impl): the stamps of its
    // last kernels land first
    if (hipDeviceSynchronize() != hipSuccess) return LH_E_HIP;
    return lh_read_stamps(out, n, reset) == hipSuccess ? LH_OK : LH_E_HIP;
}

// test hook: k_ctrl's reduced-system solve on a dense symmetric S, device pointers
// (n > LH_NPAD: k_ctrl_g's global-memory solve, the windows past LH_PMAX poses)
int lh_debug_ldlt_probe(const double* S, const double* b, int n, double* x) {
    if (!S || !b || !x) return LH_E_BADARG;
    if (n < 1 || n > 6 * LH_PMAX_WIN) return LH_E_UNSUPPORTED;
    if (n <= LH_NPAD) {
        HIPCHK(lh_launch_ldlt_probe(S, b, n, x, 0, 0.0, 0, nullptr));
    } else {
        const size_t ng = (size_t)((n + 31) & ~31);
        double* gA = nullptr;
        HIPCHK(hipMalloc(&gA, ng * ng * sizeof(double)));
        hipError_t e = lh_launch_ldlt_g_probe(S, b, n, x, gA);
        if (e == hipSuccess) e = hipDeviceSynchronize();
        (void)hipFree(gA);
        if (e != hipSuccess) return LH_E_HIP;
    }
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

// k_lin's duration per trial: after a solve, clear the stop flag, replay the trial-mode k_lin
// launch(es) `reps` times back to back between two events, raise the flag again.  Each replay reads
// the committed buffers and rewrites the candidate ones: the same work as every trial of the solve.
int lh_debug_time_lin(lh_handle* h, int reps, double* ms) {
    if (!h || !ms || reps < 1) return LH_E_BADARG;
    if (!h->uploaded) return LH_E_STATE;
    if (hipSetDevice(h->device) != hipSuccess) return LH_E_HIP;
    hipStream_t s = h->stream;
    int* done = reinterpret_cast<int*>(reinterpret_cast<char*>(h->d_ctrl.p) + offsetof(lh_ctrl, done));
    int* evo = reinterpret_cast<int*>(reinterpret_cast<char*>(h->d_ctrl.p) + offsetof(lh_ctrl, evo));
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess) return LH_E_HIP;
    if (hipEventCreate(&b) != hipSuccess) { (void)hipEventDestroy(a); return LH_E_HIP; }
    int st = LH_OK;
    const int zero = 0, one = 1;
    int evo_saved = 0;   // a solve stopped by max_iters leaves evo set: replay the full linearisation
    if (hipMemcpyAsync(&evo_saved, evo, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess) st = LH_E_HIP;
    if (st == LH_OK && hipMemcpyAsync(evo, &zero, sizeof(int), hipMemcpyHostToDevice, s) != hipSuccess) st = LH_E_HIP;
    if (st == LH_OK && hipMemcpyAsync(done, &zero, sizeof(int), hipMemcpyHostToDevice, s) != hipSuccess) st = LH_E_HIP;
    if (st == LH_OK && launch_lin(h, 1) != LH_OK) st = LH_E_HIP;   // warm-up
    if (st == LH_OK && hipEventRecord(a, s) != hipSuccess) st = LH_E_HIP;
    for (int r = 0; r < reps && st == LH_OK; ++r)
        if (launch_lin(h, 1) != LH_OK) st = LH_E_HIP;
    if (st == LH_OK && hipEventRecord(b, s) != hipSuccess) st = LH_E_HIP;
    if (hipMemcpyAsync(done, &one, sizeof(int), hipMemcpyHostToDevice, s) != hipSuccess) st = LH_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) st = LH_E_HIP;
    if (hipMemcpy(evo, &evo_saved, sizeof(int), hipMemcpyHostToDevice) != hipSuccess) st = LH_E_HIP;
    float e = 0.f;
    if (st == LH_OK && hipEventElapsedTime(&e, a, b) != hipSuccess) st = LH_E_HIP;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (st == LH_OK) *ms = (double)e / reps;
    return st;
}

int lh_debug_comm_count(lh_handle* h, int64_t* n) {
    if (!h || !n) return LH_E_BADARG;
    *n = h->n_coll;
    return LH_OK;
}

int lh_debug_chains(lh_handle* h, int* chains) {
    if (!h || !chains) return LH_E_BADARG;
    *chains = h->last_chains;
    return LH_OK;
}

int lh_debug_ladder(lh_handle* h, int* rungs, int* skipped) {
    if (!h || !rungs || !skipped) return LH_E_BADARG;
    if (!h->uploaded) return LH_E_STATE;
    *rungs = h->prm.ladder;
    *skipped = h->last_lskips;
    return LH_OK;
}

int lh_debug_batch(lh_handle* h, int* batch_max, int* batches, int* retrials) {
    if (!h || !batch_max || !batches) return LH_E_BADARG;
    if (!h->uploaded) return LH_E_STATE;
    *batch_max = h->prm.batch;
    *batches = h->last_batches;
    if (retrials) { retrials[0] = h->last_retrials[0]; retrials[1] = h->last_retrials[1]; }
    return LH_OK;
}

int lh_debug_controller(lh_handle* h, int* which) {
    if (!h || !which) return LH_E_BADARG;
    if (!h->uploaded) return LH_E_STATE;
    *which = h->P <= LH_PMAX ? 0 : h->band ? 3 : h->prm.solver == LH_SOLVER_PCG ? 2 : 1;
    if (h->band_narrow) *which |= 1 << 8;   // k_ctrl_b's one-row-per-lane back substitution
    if (h->band_lu) *which |= 1 << 9;       // k_ctrl_b's stream loaders take units (k_ctrl_b<true>)
    return LH_OK;
}

int lh_debug_mfma_probe(const double* A, const double* B, double* D) {
    if (lh_launch_mfma_probe(A, B, D) != hipSuccess) return LH_E_HIP;
    if (hipDeviceSynchronize() != hipSuccess) return LH_E_HIP;
    return LH_OK;
}

}  // extern "C"

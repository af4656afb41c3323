// lh_kernels.hip — CDNA4 (gfx950) kernels of the sliding-window BA solver.
//
// One LM trial of lego::Problem::solve (src/lego/base/problem.cpp:179-220) is
//   k_lin     landmark chunks: back-substitute the pending pose step into the
//             landmarks, evaluate chi2 at the candidate state and relinearise
//             there (residual, SE(3)/point Jacobians, Huber weights, H_pp, H_pl,
//             H_ll, b), eliminate the landmarks (Schur) — the landmark part as
//             an f64 MFMA SYRK over a chunk window — and emit one slab per chunk.
//   k_reduce  fixed-order sum of the slabs into the reduced pose system.
//   k_ctrl    one workgroup: LM accept/reject and lambda schedule
//             (isGoodStepInLM, problem.cpp:520-581), LDLT of S + lambda
//             (problem.cpp:406-420), candidate poses T' = exp(dx) T
//             (VertexPose::add, lego_types.h:61-91).
// Every reduction has a fixed order, so a solve is bitwise reproducible.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "lh_common.h"

typedef double v4d __attribute__((ext_vector_type(4)));

#define SCR_SZ 2112                  // per-wave scratch: max(64*33, 24*80) doubles
#define LMR_SZ 16                    // per-landmark slots in the per-wave landmark region
#define K_LIN_SMEM (LH_WAVES * SCR_SZ + LH_WAVES * LH_SB_LM * LMR_SZ + LH_WAVES * 16)

// Diagnostic build (-DLH_STAMPS): per-phase wave-cycle totals via s_memtime,
// summed over all waves into lh_stamps[] (cdna_hip_programming.md §7 "In-kernel
// stamps").  The product build compiles these to nothing.
#ifdef LH_STAMPS
__device__ unsigned long long lh_stamps[64];
#define STAMP_DECL unsigned long long st0_ = __builtin_amdgcn_s_memtime(), st1_;
#define STAMP(i)                                                                   \
    do {                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                         \
        st1_ = __builtin_amdgcn_s_memtime();                                       \
        if ((threadIdx.x & 63) == 0) atomicAdd(&lh_stamps[(i)], st1_ - st0_);      \
        st0_ = st1_;                                                               \
        __builtin_amdgcn_sched_barrier(0);                                         \
    } while (0)
#else
#define STAMP_DECL
#define STAMP(i)
#endif

__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)x, l);
    const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ============================================================================
// Eigen / Sophus arithmetic and the per-edge path, in the reference's
// expression order with contraction off.  This is a bitwise mirror of the
// oracle's restatement (oracle/lego_oracle.c): the Huber gate
// (base_edge.cpp:55) tests the sign of a rounding residue, so the residual
// must be computed exactly as the reference computes it.
// ============================================================================
#pragma clang fp contract(off)

// Eigen Quaternion(Matrix3): q = {w, x, y, z}, R row-major
__device__ inline void d_q_from_R(const double* R, double q[4]) {
    double t = R[0] + R[4] + R[8];
    if (t > 0.0) {
        t = sqrt(t + 1.0);
        q[0] = 0.5 * t;
        t = 0.5 / t;
        q[1] = (R[7] - R[5]) * t;
        q[2] = (R[2] - R[6]) * t;
        q[3] = (R[3] - R[1]) * t;
    } else {
        int i = 0;
        if (R[4] > R[0]) i = 1;
        if (R[8] > R[4 * i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = sqrt(R[4 * i] - R[4 * j] - R[4 * k] + 1.0);
        double c[3];
        c[i] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (R[3 * k + j] - R[3 * j + k]) * t;
        c[j] = (R[3 * j + i] + R[3 * i + j]) * t;
        c[k] = (R[3 * k + i] + R[3 * i + k]) * t;
        q[1] = c[0]; q[2] = c[1]; q[3] = c[2];
    }
}

// Eigen QuaternionBase::toRotationMatrix
__device__ inline void d_R_from_q(const double q[4], double R[9]) {
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;          R[2] = txz + twy;
    R[3] = txy + twz;          R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;          R[7] = tyz + twx;          R[8] = 1.0 - (txx + tyy);
}

__device__ __forceinline__ void d_cross(const double a[3], const double b[3], double c[3]) {
    const double c0 = a[1] * b[2] - a[2] * b[1], c1 = a[2] * b[0] - a[0] * b[2], c2 = a[0] * b[1] - a[1] * b[0];
    c[0] = c0; c[1] = c1; c[2] = c2;
}

// Eigen QuaternionBase::_transformVector (Sophus SO3 * point)
__device__ __forceinline__ void d_q_rotate(const double* q, const double v[3], double o[3]) {
    double uv[3], uv2[3];
    d_cross(q + 1, v, uv);
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    d_cross(q + 1, uv, uv2);
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = v[i] + q[0] * uv[i] + uv2[i];
}

// Eigen quaternion product + Sophus SO3Base::operator*= renormalisation
__device__ inline void d_q_mul(const double* a, const double* b, double o[4]) {
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

// Sophus SE3::exp, twist (upsilon, omega) -> (q, t)   (Sophus 1.0 se3.hpp)
__device__ inline void d_se3_exp(const double a[6], double q[4], double t[3]) {
    const double eps = 1e-10;
    const double* w = a + 3;
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const double th = sqrt(th2);
    const double half = 0.5 * th;
    double im, re;
    if (th < eps) {
        const double th4 = th2 * th2;
        im = 0.5 - (1.0 / 48.0) * th2 + (1.0 / 3840.0) * th4;
        re = 1.0 - (1.0 / 8.0) * th2 + (1.0 / 384.0) * th4;
    } else {
        im = sin(half) / th;
        re = cos(half);
    }
    q[0] = re; q[1] = im * w[0]; q[2] = im * w[1]; q[3] = im * w[2];
    double V[9];
    if (th < eps) {
        d_R_from_q(q, V);
    } else {
        const double Om[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
        double Om2[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                Om2[3 * i + j] = Om[3 * i] * Om[j] + Om[3 * i + 1] * Om[3 + j] + Om[3 * i + 2] * Om[6 + j];
        const double c1 = (1.0 - cos(th)) / th2;
        const double c2 = (th - sin(th)) / (th2 * th);
        for (int i = 0; i < 9; ++i) V[i] = ((i % 4 == 0) ? 1.0 : 0.0) + c1 * Om[i] + c2 * Om2[i];
    }
    for (int i = 0; i < 3; ++i) t[i] = V[3 * i] * a[0] + V[3 * i + 1] * a[1] + V[3 * i + 2] * a[2];
}

// estimate_ (row-major [R|t]) -> pose table entry for camera extrinsic e (LH_EXT layout)
__device__ inline void d_pose_table(const double* T12, const double* __restrict__ e, double* pt) {
    const double R[9] = {T12[0], T12[1], T12[2], T12[4], T12[5], T12[6], T12[8], T12[9], T12[10]};
    double q[4];
    d_q_from_R(R, q);                                   // SE3(estimate_)
    const double t[3] = {T12[3], T12[7], T12[11]};
    for (int i = 0; i < 4; ++i) pt[LH_PT_QT + i] = q[i];
    for (int i = 0; i < 3; ++i) pt[LH_PT_TT + i] = t[i];
    double qet[4], rt[3];
    d_q_mul(e, q, qet);                                 // _cam_ext * T
    d_q_rotate(e, t, rt);
    for (int i = 0; i < 4; ++i) pt[LH_PT_QET + i] = qet[i];
    for (int i = 0; i < 3; ++i) pt[LH_PT_TET + i] = e[4 + i] + rt[i];
    double Rt[9];
    d_R_from_q(q, Rt);                                  // T.rotationMatrix()
    for (int i = 0; i < 9; ++i) pt[LH_PT_RT + i] = Rt[i];
    pt[23] = 0.0;
}

struct EdgeEval {
    double r0, r1, e2, rho0, rho1, rho2;
    double W00, W01, W10, W11;
    double Jp[12];   // 2 x 6, translation-first twist (lego_types.h:246-248)
    double Jl[6];    // 2 x 3
};

// residual_ = z - pi(K (ext (T X))), pi(q) = q / (q_z + 1e-18)   (lego_types.h:200-216)
__device__ __forceinline__ void edge_residual(const double* __restrict__ pt, const double* __restrict__ e, bool ext_id,
                                              const double X[3], double u, double v, const lh_params& prm,
                                              double& r0, double& r1) {
    double Pb[3], Pc[3];
    d_q_rotate(pt + LH_PT_QT, X, Pb);
#pragma unroll
    for (int i = 0; i < 3; ++i) Pb[i] = Pb[i] + pt[LH_PT_TT + i];
    if (ext_id) {
#pragma unroll
        for (int i = 0; i < 3; ++i) Pc[i] = Pb[i];       // identity quaternion and zero t: exact
    } else {
        d_q_rotate(e, Pb, Pc);
#pragma unroll
        for (int i = 0; i < 3; ++i) Pc[i] = Pc[i] + e[4 + i];
    }
    const double fx = prm.K[0], fy = prm.K[1], cx = prm.K[2], cy = prm.K[3];
    double p0 = fx * Pc[0] + cx * Pc[2];                  // + 0 * Pc[1]: exact
    double p1 = fy * Pc[1] + cy * Pc[2];
    const double den = Pc[2] + 1e-18;
    p0 /= den;
    p1 /= den;
    r0 = u - p0;
    r1 = v - p1;
}

// HuberCost::compute (cost_function.cpp:5-17) + computeRobustInformation (base_edge.cpp:44-64)
__device__ __forceinline__ void edge_robust(EdgeEval& E, const lh_params& prm) {
    E.e2 = E.r0 * E.r0 + E.r1 * E.r1;
    const double delta = prm.huber_delta;
    if (delta > 0.0) {
        const double d2 = delta * delta;
        if (E.e2 <= d2) {
            E.rho0 = E.e2; E.rho1 = 1.0; E.rho2 = 0.0;
        } else {
            const double s = sqrt(E.e2);
            E.rho0 = 2 * s * delta - d2;
            E.rho1 = delta / s;
            E.rho2 = -0.5 * E.rho1 / E.e2;
        }
        E.W00 = E.rho1; E.W01 = 0.0; E.W10 = 0.0; E.W11 = E.rho1;
        if (E.rho1 + 2 * E.rho2 * E.e2 > 0.0) {
            const double s2 = 2 * E.rho2;
            E.W00 += s2 * E.r0 * E.r0;
            E.W01 += s2 * E.r0 * E.r1;
            E.W10 += s2 * E.r1 * E.r0;
            E.W11 += s2 * E.r1 * E.r1;
        }
    } else {
        E.rho0 = E.e2; E.rho1 = 1.0; E.rho2 = 0.0;
        E.W00 = 1.0; E.W01 = 0.0; E.W10 = 0.0; E.W11 = 1.0;
    }
}

// EdgeProjection::computeJacobians (lego_types.h:218-254) at Pc = (ext T) X
__device__ __forceinline__ void edge_jacobians(const double* __restrict__ pt, const double* __restrict__ e, bool ext_id,
                                               const double X[3], const lh_params& prm, double Jp[12], double Jl[6]) {
    double Pc[3];
    d_q_rotate(pt + LH_PT_QET, X, Pc);
#pragma unroll
    for (int i = 0; i < 3; ++i) Pc[i] = Pc[i] + pt[LH_PT_TET + i];
    const double fx = prm.K[0], fy = prm.K[1];
    const double x = Pc[0], y = Pc[1], z = Pc[2];
    const double zi = 1.0 / (z + 1e-18);
    const double zi2 = zi * zi;
    Jp[0] = -fx * zi;              Jp[1] = 0.0;                  Jp[2] = fx * x * zi2;
    Jp[3] = fx * x * y * zi2;      Jp[4] = -fx - fx * x * x * zi2; Jp[5] = fx * y * zi;
    Jp[6] = 0.0;                   Jp[7] = -fy * zi;             Jp[8] = fy * y * zi2;
    Jp[9] = fy + fy * y * y * zi2; Jp[10] = -fy * x * y * zi2;   Jp[11] = -fy * x * zi;
    // j_j = (j_i(:, 0:3) * ext.rotationMatrix()) * T.rotationMatrix()
    double A[6];
    if (ext_id) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) A[3 * i + j] = Jp[6 * i + j];   // J * I: exact
    } else {
        const double* Re = e + 7;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                A[3 * i + j] = Jp[6 * i] * Re[j] + Jp[6 * i + 1] * Re[3 + j] + Jp[6 * i + 2] * Re[6 + j];
    }
    const double* Rt = pt + LH_PT_RT;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            Jl[3 * i + j] = A[3 * i] * Rt[j] + A[3 * i + 1] * Rt[3 + j] + A[3 * i + 2] * Rt[6 + j];
}

#pragma clang fp contract(fast)

// ============================================================================
// k_lin: one workgroup (4 waves) per landmark chunk; one sub-batch (<= 8
// landmarks, <= 64 observations, one observation per lane) per wave at a time.
// ============================================================================
template <int T>
struct LinCfg {
    static constexpr int NT = T * (T + 1) / 2;          // upper MFMA tiles of the window
    static constexpr int GS = (T == 1) ? 16 : (T == 4 ? 80 : 48);  // G row stride: 16T + pad, conflict-free b64 frag loads
    static constexpr int UMAX = (16 * T) / 6;           // window poses that fit 16T rows
    static constexpr int NTASK = (UMAX * LH_TASKS + 63) / 64;
};

template <int T, bool TRIAL>
__global__ __launch_bounds__(256, 2) void k_lin(
    const lh_chunk* __restrict__ chunks, const lh_subbatch* __restrict__ sbs, const uint32_t* __restrict__ lm_ptr,
    const double* __restrict__ obs_uv, const uint32_t* __restrict__ obs_meta, double* __restrict__ Xbuf,
    double* __restrict__ cache, const double* __restrict__ ptab, const double* __restrict__ ext,
    const lh_ctrl* __restrict__ ctrl, const double* __restrict__ dxp, double* __restrict__ edge_rho,
    double* __restrict__ slabs, lh_params prm, int L, uint32_t fixed_mask, int chunk_base) {
    using Cfg = LinCfg<T>;
    __shared__ __attribute__((aligned(16))) double smem[K_LIN_SMEM];

    if (__builtin_amdgcn_readfirstlane(ctrl->done)) return;
    const int cur = __builtin_amdgcn_readfirstlane(ctrl->cur);
    const int cand = 1 - cur;
    const double lambda = ctrl->lambda;
    const int chunk = chunk_base + blockIdx.x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const lh_chunk ck = chunks[chunk];
    const int PT = prm.P * prm.ncam * LH_PT;

    double* scr = smem + wave * SCR_SZ;
    double* lmr = smem + LH_WAVES * SCR_SZ + wave * (LH_SB_LM * LMR_SZ);
    uint64_t* masks = reinterpret_cast<uint64_t*>(smem + LH_WAVES * SCR_SZ + LH_WAVES * LH_SB_LM * LMR_SZ) + wave * 16;

    const double* Xc = Xbuf + (size_t)cur * L * 3;
    double* Xn = Xbuf + (size_t)cand * L * 3;
    const double* cc = cache + (size_t)cur * L * LH_CACHE;
    double* cn = cache + (size_t)cand * L * LH_CACHE;
    const double* ptc = ptab + (size_t)cur * PT;
    const double* ptn = ptab + (size_t)cand * PT;

    v4d acc[Cfg::NT];
#pragma unroll
    for (int t = 0; t < Cfg::NT; ++t) acc[t] = v4d{0.0, 0.0, 0.0, 0.0};
    double task[Cfg::NTASK];
#pragma unroll
    for (int m = 0; m < Cfg::NTASK; ++m) task[m] = 0.0;
    double chi_acc = 0.0, scale_acc = 0.0, maxd = 0.0, ndeg = 0.0;
    const int U = ck.U;
    STAMP_DECL

    for (int sb = ck.sb_begin + wave; sb < (int)ck.sb_end; sb += LH_WAVES) {
        const lh_subbatch S = sbs[sb];
        const int nobs = S.n_obs, nlm = S.n_lm;
        const bool has = lane < nobs;
        const int o = S.obs_begin + lane;
        const uint32_t meta = has ? obs_meta[o] : 0u;
        const int p = LH_META_POSE(meta), cam = LH_META_CAM(meta), slot = LH_META_SLOT(meta), ls = LH_META_LMS(meta);
        const bool pfixed = (fixed_mask >> p) & 1u;
        const int lm = S.lm_begin + ls;
        double X[3] = {0.0, 0.0, 0.0};
        double u = 0.0, v = 0.0;
        if (has) {
            u = obs_uv[2 * (size_t)o];
            v = obs_uv[2 * (size_t)o + 1];
            X[0] = Xc[3 * (size_t)lm]; X[1] = Xc[3 * (size_t)lm + 1]; X[2] = Xc[3 * (size_t)lm + 2];
        }
        const double* e = ext + cam * LH_EXT;
        const bool ext_id = (prm.ext_identity >> cam) & 1;

        // ---- back-substitution of the pending pose step (problem.cpp:426-429) ----
        if (TRIAL) {
            double v3[3] = {0.0, 0.0, 0.0};
            if (has && !pfixed) {
                const double* pt = ptc + (p * prm.ncam + cam) * LH_PT;
                EdgeEval E;
                edge_residual(pt, e, ext_id, X, u, v, prm, E.r0, E.r1);
                edge_robust(E, prm);
                edge_jacobians(pt, e, ext_id, X, prm, E.Jp, E.Jl);
                const double* d = dxp + 6 * p;
                double jd0 = 0.0, jd1 = 0.0;
#pragma unroll
                for (int a = 0; a < 6; ++a) { jd0 += E.Jp[a] * d[a]; jd1 += E.Jp[6 + a] * d[a]; }
                double y0 = E.W00 * jd0 + E.W01 * jd1, y1 = E.W10 * jd0 + E.W11 * jd1;
#pragma unroll
                for (int c = 0; c < 3; ++c) v3[c] = E.Jl[c] * y0 + E.Jl[3 + c] * y1;
            }
            scr[3 * lane] = v3[0]; scr[3 * lane + 1] = v3[1]; scr[3 * lane + 2] = v3[2];
            wave_sync();
            if (lane < nlm) {
                const int lmj = S.lm_begin + lane;
                const int i0 = (int)(lm_ptr[lmj] - S.obs_begin), i1 = (int)(lm_ptr[lmj + 1] - S.obs_begin);
                double s0 = 0.0, s1 = 0.0, s2 = 0.0;
                for (int i = i0; i < i1; ++i) { s0 += scr[3 * i]; s1 += scr[3 * i + 1]; s2 += scr[3 * i + 2]; }
                const double* cl = cc + (size_t)lmj * LH_CACHE;
                const double l00 = cl[0], l10 = cl[1], l11 = cl[2], l20 = cl[3], l21 = cl[4], l22 = cl[5];
                const double b0 = cl[6], b1 = cl[7], b2 = cl[8];
                double t0 = b0 - s0, t1 = b1 - s1, t2 = b2 - s2;
                double y0 = t0 / l00, y1 = (t1 - l10 * y0) / l11, y2 = (t2 - l20 * y0 - l21 * y1) / l22;
                double d2 = y2 / l22, d1 = (y1 - l21 * d2) / l11, d0 = (y0 - l10 * d1 - l20 * d2) / l00;
                if (prm.guard && !(l00 == l00)) { d0 = d1 = d2 = 0.0; }   // skipped degenerate landmark
                double sc;
                if (prm.strategy == 0) sc = d0 * (lambda * d0 + b0) + d1 * (lambda * d1 + b1) + d2 * (lambda * d2 + b2);
                else sc = d0 * (lambda * cl[9] * d0 + b0) + d1 * (lambda * cl[10] * d1 + b1) + d2 * (lambda * cl[11] * d2 + b2);
                scale_acc += sc;
                const double x0 = Xc[3 * (size_t)lmj], x1 = Xc[3 * (size_t)lmj + 1], x2 = Xc[3 * (size_t)lmj + 2];
                double n0 = x0, n1 = x1, n2 = x2;
                if (isfinite(d0) && isfinite(d1) && isfinite(d2)) { n0 = x0 + d0; n1 = x1 + d1; n2 = x2 + d2; }   // VertexXYZ::add
                Xn[3 * (size_t)lmj] = n0; Xn[3 * (size_t)lmj + 1] = n1; Xn[3 * (size_t)lmj + 2] = n2;
                lmr[LMR_SZ * lane] = n0; lmr[LMR_SZ * lane + 1] = n1; lmr[LMR_SZ * lane + 2] = n2;
            }
            wave_sync();
            if (has) { X[0] = lmr[LMR_SZ * ls]; X[1] = lmr[LMR_SZ * ls + 1]; X[2] = lmr[LMR_SZ * ls + 2]; }
        } else {
            if (lane < nlm) {
                const int lmj = S.lm_begin + lane;
                Xn[3 * (size_t)lmj] = Xc[3 * (size_t)lmj];
                Xn[3 * (size_t)lmj + 1] = Xc[3 * (size_t)lmj + 1];
                Xn[3 * (size_t)lmj + 2] = Xc[3 * (size_t)lmj + 2];
            }
        }

        STAMP(0);
        // ---- evaluate and linearise at the candidate (problem.cpp:285-331, :523-526) ----
        double hll[6] = {0, 0, 0, 0, 0, 0}, bl[3] = {0, 0, 0};
        double hpp[21], bp[6], hpl[18];
#pragma unroll
        for (int i = 0; i < 21; ++i) hpp[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) bp[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 18; ++i) hpl[i] = 0.0;
        if (has) {
            const double* pt = ptn + (p * prm.ncam + cam) * LH_PT;
            EdgeEval E;
            edge_residual(pt, e, ext_id, X, u, v, prm, E.r0, E.r1);
            edge_robust(E, prm);
            edge_jacobians(pt, e, ext_id, X, prm, E.Jp, E.Jl);
            edge_rho[o] = E.rho0;
            chi_acc += E.rho0;
            const double dr = (prm.huber_delta > 0.0) ? E.rho1 : 1.0;
            double WJl[6], WJp[12];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                WJl[c] = E.W00 * E.Jl[c] + E.W01 * E.Jl[3 + c];
                WJl[3 + c] = E.W10 * E.Jl[c] + E.W11 * E.Jl[3 + c];
            }
            hll[0] = E.Jl[0] * WJl[0] + E.Jl[3] * WJl[3];
            hll[1] = E.Jl[0] * WJl[1] + E.Jl[3] * WJl[4];
            hll[2] = E.Jl[0] * WJl[2] + E.Jl[3] * WJl[5];
            hll[3] = E.Jl[1] * WJl[1] + E.Jl[4] * WJl[4];
            hll[4] = E.Jl[1] * WJl[2] + E.Jl[4] * WJl[5];
            hll[5] = E.Jl[2] * WJl[2] + E.Jl[5] * WJl[5];
#pragma unroll
            for (int c = 0; c < 3; ++c) bl[c] = -((dr * E.Jl[c]) * E.r0 + (dr * E.Jl[3 + c]) * E.r1);
            if (!pfixed) {
#pragma unroll
                for (int a = 0; a < 6; ++a) {
                    WJp[a] = E.W00 * E.Jp[a] + E.W01 * E.Jp[6 + a];
                    WJp[6 + a] = E.W10 * E.Jp[a] + E.W11 * E.Jp[6 + a];
                }
                int k = 0;
#pragma unroll
                for (int a = 0; a < 6; ++a)
#pragma unroll
                    for (int b = a; b < 6; ++b) hpp[k++] = E.Jp[a] * WJp[b] + E.Jp[6 + a] * WJp[6 + b];
#pragma unroll
                for (int a = 0; a < 6; ++a) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) hpl[3 * a + c] = E.Jp[a] * WJl[c] + E.Jp[6 + a] * WJl[3 + c];
                    bp[a] = -((dr * E.Jp[a]) * E.r0 + (dr * E.Jp[6 + a]) * E.r1);
                }
            }
        }

        STAMP(1);
        // ---- per-landmark H_ll, b_l; Cholesky; cache for the next back-substitution ----
        wave_sync();
#pragma unroll
        for (int i = 0; i < 6; ++i) scr[9 * lane + i] = hll[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) scr[9 * lane + 6 + i] = bl[i];
        wave_sync();
        if (lane < nlm) {
            const int lmj = S.lm_begin + lane;
            const int i0 = (int)(lm_ptr[lmj] - S.obs_begin), i1 = (int)(lm_ptr[lmj + 1] - S.obs_begin);
            double h[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            for (int i = i0; i < i1; ++i)
#pragma unroll
                for (int j = 0; j < 9; ++j) h[j] += scr[9 * i + j];
            maxd = fmax(maxd, fmax(fabs(h[0]), fmax(fabs(h[3]), fabs(h[5]))));
            double l00 = sqrt(h[0]);
            double l10 = h[1] / l00, l20 = h[2] / l00;
            double a11 = h[3] - l10 * l10;
            double l11 = sqrt(a11);
            double l21 = (h[4] - l20 * l10) / l11;
            double a22 = h[5] - l20 * l20 - l21 * l21;
            double l22 = sqrt(a22);
            const bool pd = (h[0] > 0.0) && (a11 > 0.0) && (a22 > 0.0) && isfinite(l22) && isfinite(l21);
            if (!pd) {
                ndeg += 1.0;
                l00 = __builtin_nan("");   // poisons the Schur step, as a singular LU inverse does (problem.cpp:399)
            }
            double w0 = h[6] / l00, w1 = (h[7] - l10 * w0) / l11, w2 = (h[8] - l20 * w0 - l21 * w1) / l22;
            double* cl = cn + (size_t)lmj * LH_CACHE;
            cl[0] = l00; cl[1] = l10; cl[2] = l11; cl[3] = l20; cl[4] = l21; cl[5] = l22;
            cl[6] = h[6]; cl[7] = h[7]; cl[8] = h[8];
            cl[9] = h[0]; cl[10] = h[3]; cl[11] = h[5];
            double* lr = lmr + LMR_SZ * lane;
            lr[3] = l00; lr[4] = l10; lr[5] = l11; lr[6] = l20; lr[7] = l21; lr[8] = l22;
            lr[9] = w0; lr[10] = w1; lr[11] = w2;
            lr[12] = pd ? 1.0 : 0.0;
        }
        wave_sync();

        STAMP(2);
        // ---- per observation: G = H_pl L^-T and bsd = G w = H_pl H_ll^-1 b_l ----
        double G[18], bsd[6];
#pragma unroll
        for (int i = 0; i < 18; ++i) G[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) bsd[i] = 0.0;
        if (has && !pfixed) {
            const double* lr = lmr + LMR_SZ * ls;
            const double l00 = lr[3], l10 = lr[4], l11 = lr[5], l20 = lr[6], l21 = lr[7], l22 = lr[8];
            const double w0 = lr[9], w1 = lr[10], w2 = lr[11];
            const bool skip = prm.guard && lr[12] == 0.0;
            if (!skip) {
#pragma unroll
                for (int a = 0; a < 6; ++a) {
                    double g0 = hpl[3 * a] / l00;
                    double g1 = (hpl[3 * a + 1] - l10 * g0) / l11;
                    double g2 = (hpl[3 * a + 2] - l20 * g0 - l21 * g1) / l22;
                    G[3 * a] = g0; G[3 * a + 1] = g1; G[3 * a + 2] = g2;
                    bsd[a] = g0 * w0 + g1 * w1 + g2 * w2;
                }
            }
        }

        STAMP(3);
        // ---- per-pose sums (H_pp, b_p, bsd) in ascending lane order ----
#pragma unroll
        for (int i = 0; i < 21; ++i) scr[LH_TASKS * lane + i] = hpp[i];
#pragma unroll
        for (int i = 0; i < 6; ++i) scr[LH_TASKS * lane + 21 + i] = bp[i];
#pragma unroll
        for (int i = 0; i < 6; ++i) scr[LH_TASKS * lane + 27 + i] = bsd[i];
        for (int uu = 0; uu < U; ++uu) {
            uint64_t mk = __ballot(has && slot == uu);
            if (lane == 0) masks[uu] = mk;
        }
        wave_sync();
#pragma unroll
        for (int m = 0; m < Cfg::NTASK; ++m) {
            const int t = lane + 64 * m;
            if (t < U * LH_TASKS) {
                const int uu = t / LH_TASKS, ee = t - uu * LH_TASKS;
                uint64_t mk = masks[uu];
                double s = task[m];
                while (mk) {
                    const int i = __builtin_ctzll(mk);
                    s += scr[LH_TASKS * i + ee];
                    mk &= mk - 1;
                }
                task[m] = s;
            }
        }
        wave_sync();

        STAMP(4);
        // ---- G rows into the window image [k][16T], then the MFMA SYRK ----
        {
            double2* z = reinterpret_cast<double2*>(scr);
            const int nz = (3 * LH_SB_LM * Cfg::GS) / 2;
            for (int i = lane; i < nz; i += 64) z[i] = double2{0.0, 0.0};
        }
        wave_sync();
        if (has) {
#pragma unroll
            for (int a = 0; a < 6; ++a)
#pragma unroll
                for (int j = 0; j < 3; ++j) scr[(3 * ls + j) * Cfg::GS + 6 * slot + a] = G[3 * a + j];
        }
        wave_sync();
        STAMP(5);
        const int nk = (3 * nlm + 3) >> 2;
        for (int s = 0; s < nk; ++s) {
            double f[T];
            const double* row = scr + (4 * s + (lane >> 4)) * Cfg::GS + (lane & 15);
#pragma unroll
            for (int R = 0; R < T; ++R) f[R] = row[16 * R];
            int t = 0;
#pragma unroll
            for (int R = 0; R < T; ++R)
#pragma unroll
                for (int Cc = R; Cc < T; ++Cc) {
                    acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(f[R], f[Cc], acc[t], 0, 0, 0);
                    ++t;
                }
        }
        wave_sync();
        STAMP(6);
    }

    // ---- combine the 4 waves in fixed order and write the chunk slab ----
    __syncthreads();
    double* sl = smem;   // reuses the scratch (SLAB_STRIDE <= 4 * SCR_SZ)
    const int ntile = Cfg::NT * 256;
    const int ntask = U * LH_TASKS;
    // wave-level scalar reductions (fixed butterfly)
    for (int off = 32; off > 0; off >>= 1) {
        chi_acc += __shfl_xor(chi_acc, off);
        scale_acc += __shfl_xor(scale_acc, off);
        ndeg += __shfl_xor(ndeg, off);
        maxd = fmax(maxd, __shfl_xor(maxd, off));
    }
    for (int w = 0; w < LH_WAVES; ++w) {
        if (wave == w) {
#pragma unroll
            for (int t = 0; t < Cfg::NT; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int idx = t * 256 + ((lane >> 4) + 4 * i) * 16 + (lane & 15);
                    sl[idx] = (w == 0 ? 0.0 : sl[idx]) + acc[t][i];
                }
#pragma unroll
            for (int m = 0; m < Cfg::NTASK; ++m) {
                const int t = lane + 64 * m;
                if (t < ntask) sl[LH_SLAB_TASK_OFF + t] = (w == 0 ? 0.0 : sl[LH_SLAB_TASK_OFF + t]) + task[m];
            }
            if (lane == 0) {
                double* sc = sl + LH_SLAB_SC_OFF;
                if (w == 0) { sc[0] = chi_acc; sc[1] = scale_acc; sc[2] = ndeg; sc[3] = maxd; }
                else { sc[0] += chi_acc; sc[1] += scale_acc; sc[2] += ndeg; sc[3] = fmax(sc[3], maxd); }
            }
        }
        __syncthreads();
    }
    double* gs = slabs + (size_t)chunk * LH_SLAB_STRIDE;
    for (int i = tid; i < ntile; i += 256) gs[i] = sl[i];
    for (int i = tid; i < ntask; i += 256) gs[LH_SLAB_TASK_OFF + i] = sl[LH_SLAB_TASK_OFF + i];
    if (tid < 4) gs[LH_SLAB_SC_OFF + tid] = sl[LH_SLAB_SC_OFF + tid];
    STAMP(7);
}

// ============================================================================
// k_reduce: fixed-order sum of chunk slabs into the reduced pose system.
// Block b < npairs handles pose pair (pp[b], pq[b]); block npairs the scalars.
// ============================================================================
__device__ __forceinline__ int hpp_index(int a, int b) {   // packed upper 6x6, a <= b
    return a * 6 - (a * (a - 1)) / 2 + (b - a);
}

#define RT 1024
#define RW (RT / 64)

__global__ __launch_bounds__(RT) void k_reduce(const double* __restrict__ slabs, const uint32_t* __restrict__ pair_ptr,
                                               const uint32_t* __restrict__ items, const uint16_t* __restrict__ pair_pq,
                                               const lh_ctrl* __restrict__ ctrl, double* __restrict__ rs,
                                               double* __restrict__ maxd_out, lh_params prm, int n_chunks) {
    if (__builtin_amdgcn_readfirstlane(ctrl->done)) return;
    STAMP_DECL
    __shared__ double part[3][RW][64];
    const lh_rs_layout LY = lh_rs_make(prm.P);
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (b == LY.npairs) {
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, mx = 0.0;
        for (int c = tid; c < n_chunks; c += RT) {
            const double* sc = slabs + (size_t)c * LH_SLAB_STRIDE + LH_SLAB_SC_OFF;
            s0 += sc[0]; s1 += sc[1]; s2 += sc[2]; mx = fmax(mx, sc[3]);
        }
        for (int off = 32; off > 0; off >>= 1) {
            s0 += __shfl_xor(s0, off); s1 += __shfl_xor(s1, off); s2 += __shfl_xor(s2, off);
            mx = fmax(mx, __shfl_xor(mx, off));
        }
        if (lane == 0) { part[0][wave][0] = s0; part[1][wave][0] = s1; part[2][wave][0] = s2; part[0][wave][1] = mx; }
        __syncthreads();
        if (tid == 0) {
            double a0 = 0.0, a1 = 0.0, a2 = 0.0, m = 0.0;
            for (int w = 0; w < RW; ++w) { a0 += part[0][w][0]; a1 += part[1][w][0]; a2 += part[2][w][0]; m = fmax(m, part[0][w][1]); }
            rs[LY.off_sc + LH_SC_CHI2] = a0;
            rs[LY.off_sc + LH_SC_SCALE] = a1;
            rs[LY.off_sc + LH_SC_NDEG] = a2;
            rs[LY.off_sc + LH_SC_MAXD] = m;
            *maxd_out = m;
        }
        return;
    }
    const int p = pair_pq[2 * b], q = pair_pq[2 * b + 1];
    const bool diag = p == q;
    const int a = lane / 6, bb = lane - 6 * (lane / 6);
    // lanes 0..35: S entry (a, bb) [+ H_pp entry on the diagonal]; 36..41: b_p; 42..47: bsd
    int off_s = 0, off_h = 0;
    if (lane < 36) off_h = LH_SLAB_TASK_OFF + (diag ? ((a < bb ? a : bb) * 6 - ((a < bb ? a : bb) * ((a < bb ? a : bb) - 1)) / 2 + ((a < bb ? bb : a) - (a < bb ? a : bb))) : 0);
    else if (lane < 42) off_h = LH_SLAB_TASK_OFF + 21 + (lane - 36);
    else if (lane < 48) off_h = LH_SLAB_TASK_OFF + 27 + (lane - 42);
    const bool act_s = lane < 36, act_h = (lane < 36 && diag) || (lane >= 36 && lane < 48 && diag);
    double vs = 0.0, vh = 0.0;
    const int it0 = pair_ptr[b], it1 = pair_ptr[b + 1];
    for (int it = it0 + wave; it < it1; it += RW) {
        const uint32_t item = items[it];
        const int ch = item >> 11, T = (item >> 8) & 7, sp = (item >> 4) & 15, sq = item & 15;
        const double* sl = slabs + (size_t)ch * LH_SLAB_STRIDE;
        if (act_s) {
            int ra = 6 * sp + a, rc = 6 * sq + bb;
            if ((ra >> 4) > (rc >> 4)) { const int t = ra; ra = rc; rc = t; }
            const int R = ra >> 4, Cc = rc >> 4;
            off_s = (R * T - (R * (R - 1)) / 2 + (Cc - R)) * 256 + (ra & 15) * 16 + (rc & 15);
            vs += sl[off_s];
        }
        if (act_h) vh += sl[off_h + sp * LH_TASKS];
    }
    part[0][wave][lane] = vs;
    part[1][wave][lane] = vh;
    __syncthreads();
    if (wave == 0) {
        double s = 0.0, h = 0.0;
        for (int w = 0; w < RW; ++w) { s += part[0][w][lane]; h += part[1][w][lane]; }
        if (lane < 36) {
            rs[LY.off_S + b * 36 + lane] = (diag ? h : 0.0) - s;
            if (diag && a == bb) rs[LY.off_hd + 6 * p + a] = h;
        }
        // b_p (lanes 36..41) and bs = b_p - bsd (needs lane + 6)
        const double bsd = __shfl_down(h, 6);
        if (diag && lane >= 36 && lane < 42) {
            rs[LY.off_bp + 6 * p + (lane - 36)] = h;
            rs[LY.off_bs + 6 * p + (lane - 36)] = h - bsd;
        }
    }
    STAMP(20);
}

// ============================================================================
// k_ctrl: LM controller + reduced-system solve, one workgroup of 256 threads.
// ============================================================================
#define CT 256
#define AS (LH_NPAD + 1)   // LDS row stride of the reduced matrix (odd: conflict-free column reads)

__device__ inline double rs_S(const double* __restrict__ rs, const lh_rs_layout& LY, int P, int i, int j) {
    int pi = i / 6, pj = j / 6, a = i - 6 * pi, b = j - 6 * pj;
    if (pi > pj) { int t = pi; pi = pj; pj = t; t = a; a = b; b = t; }
    const int pair = pi * P - (pi * (pi - 1)) / 2 + (pj - pi);
    return rs[LY.off_S + pair * 36 + a * 6 + b];
}

__global__ __launch_bounds__(CT) void k_ctrl(lh_ctrl* __restrict__ ctrl, double* __restrict__ rs_commit,
                                             const double* __restrict__ rs_stage, const double* __restrict__ maxd_in,
                                             double* __restrict__ pose_mat, double* __restrict__ ptab,
                                             const double* __restrict__ ext, double* __restrict__ dxp, lh_params prm,
                                             int mode /* 0 init, 1 trial */, volatile int* __restrict__ host_done) {
    __shared__ double A[LH_NPAD * AS];
    __shared__ double Xp[LH_NPAD * 8];     // unscaled panel column values
    __shared__ double Dv[LH_NPAD], yv[LH_NPAD], dg[LH_NPAD];
    __shared__ int perm[LH_NPAD];
    __shared__ int s_flags[4];
    __shared__ double s_red[CT / 64];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int P = prm.P, n = 6 * P;
    const lh_rs_layout LY = lh_rs_make(P);
    STAMP_DECL

    // ---------------- LM bookkeeping (one thread) ----------------
    if (tid == 0) {
        lh_ctrl& c = *ctrl;
        int accept_copy = 0;
        if (!c.done) {
            const double tchi = 0.5 * rs_stage[LY.off_sc + LH_SC_CHI2];
            if (mode == 0) {
                // computeLambdaInitLM (problem.cpp:470-504)
                c.ni = 2.0;
                c.chi = tchi;
                c.chi2_initial = tchi;
                if (prm.strategy == 0) {
                    if (!prm.lambda_given) {
                        double m = 0.0;
                        for (int i = 0; i < n; ++i) m = fmax(fabs(rs_stage[LY.off_hd + i]), m);
                        m = fmax(*maxd_in, m);
                        m = fmin(prm.lambda_cap, m);
                        c.lambda = prm.tau * m;
                    } else {
                        c.lambda = prm.lambda_init;
                    }
                } else {
                    c.lambda = 1e-5;
                }
                c.last_chi = 1e20;
                c.iter = 0; c.false_cnt = 0; c.trials = 0; c.accepted = 0; c.trace_len = 0;
                c.cur = 1 - c.cur;     // the initial linearisation becomes the committed one
                accept_copy = 1;
                if (prm.max_iters <= 0) c.done = 1;
                else { c.trace_chi[0] = c.chi; c.trace_lambda[0] = c.lambda; c.trace_len = 1; }
            } else {
                // isGoodStepInLM (problem.cpp:520-581)
                bool ok;
                const double sl = rs_stage[LY.off_sc + LH_SC_SCALE];
                if (prm.strategy == 0) {
                    double scale = 0.5 * (c.spose + sl);
                    scale += 1e-10;
                    const double rho = (c.chi - tchi) / scale;
                    ok = rho > 0 && isfinite(tchi);
                    if (ok) {
                        double alpha = 1.0 - pow((2 * rho - 1), 3);
                        alpha = fmin(alpha, 2.0 / 3.0);
                        c.lambda *= fmax(1.0 / 3.0, alpha);
                        c.ni = 2;
                        c.chi = tchi;
                    } else {
                        c.lambda *= c.ni;
                        c.ni *= 2;
                    }
                } else {
                    double scale = 0.5 * (c.spose + sl);
                    scale += 1e-10;
                    const double rho = (c.chi - tchi) / scale;
                    ok = rho > 0 && isfinite(tchi);
                    if (ok) { c.lambda = fmax(c.lambda / 9.0, 1e-7); c.chi = tchi; }
                    else c.lambda = fmin(c.lambda * 11.0, 1e7);
                }
                c.trials += 1;
                bool inner_end = false;
                if (ok) {
                    c.accepted += 1;
                    c.cur = 1 - c.cur;   // commit candidate landmarks, caches and poses
                    accept_copy = 1;
                    c.false_cnt = 0;
                    inner_end = true;
                } else {
                    c.false_cnt += 1;    // rollbackStates: the committed buffers are untouched
                    inner_end = c.false_cnt >= prm.max_trials;
                }
                if (inner_end) {
                    c.iter += 1;
                    if (c.last_chi - c.chi < prm.stop_dchi2) c.done = 1;
                    c.last_chi = c.chi;
                    if (!c.done && c.iter >= prm.max_iters) c.done = 1;
                    if (!c.done) {
                        c.false_cnt = 0;
                        if (c.trace_len < LH_TRACE) {
                            c.trace_chi[c.trace_len] = c.chi;
                            c.trace_lambda[c.trace_len] = c.lambda;
                        }
                        c.trace_len += 1;
                    }
                }
            }
        }
        s_flags[0] = c.done;
        s_flags[1] = accept_copy;
        s_flags[2] = c.cur;
        if (c.done && host_done) *host_done = 1;
    }
    __syncthreads();
    const int done = s_flags[0], cur = s_flags[2];
    if (s_flags[1]) {
        for (int i = tid; i < LY.total; i += CT) rs_commit[i] = rs_stage[i];
        __syncthreads();
    }
    if (done) return;
    STAMP(10);
    const double lambda = ctrl->lambda;
    const double* rs = rs_commit;

    // ---------------- (S + lambda D) with Eigen's LDLT pivot order ----------------
    // Eigen LDLT (left-looking) pivots on the largest remaining original
    // diagonal: the order of |diag| descending (problem.cpp:420).
    for (int i = tid; i < n; i += CT) {
        double d = rs_S(rs, LY, P, i, i);
        d = (prm.strategy == 0) ? d + lambda : d + lambda * d;
        dg[i] = d;
    }
    __syncthreads();
    for (int i = tid; i < n; i += CT) {
        // total order (NaN last, ties by index) so perm is a permutation even for a poisoned S
        double di = fabs(dg[i]);
        if (!(di == di)) di = -1.0;
        int r = 0;
        for (int j = 0; j < n; ++j) {
            double dj = fabs(dg[j]);
            if (!(dj == dj)) dj = -1.0;
            r += (dj > di) || (dj == di && j < i);
        }
        perm[r] = i;
    }
    __syncthreads();
    for (int idx = tid; idx < n * n; idx += CT) {
        const int r = idx / n, s = idx - r * n;
        if (s > r) continue;
        const int i = perm[r], j = perm[s];
        A[r * AS + s] = (r == s) ? dg[i] : rs_S(rs, LY, P, i, j);
    }
    for (int i = tid; i < n; i += CT) yv[i] = rs[LY.off_bs + perm[i]];
    __syncthreads();

    STAMP(11);
    // ---------------- blocked right-looking LDL^T, panel width 8 ----------------
    for (int k0 = 0; k0 < n; k0 += 8) {
        const int kb = min(8, n - k0);
        if (wave == 0) {
            // panel rows k0 + lane and k0 + 64 + lane, columns k0..k0+kb-1, in registers
            double p0[8], p1[8];
            const int i0 = k0 + lane, i1 = k0 + 64 + lane;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                p0[c] = (c < kb && i0 < n && c <= lane) ? A[i0 * AS + k0 + c] : 0.0;
                p1[c] = (c < kb && i1 < n) ? A[i1 * AS + k0 + c] : 0.0;
            }
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                if (c < kb) {
                    const double d = readlane_d(p0[c], c);
                    const double inv = (d != 0.0) ? 1.0 / d : 0.0;
                    const double x0 = p0[c], x1 = p1[c];
                    if (lane == 0) Dv[k0 + c] = d;
                    if (i0 < n) Xp[i0 * 8 + c] = x0;
                    if (i1 < n) Xp[i1 * 8 + c] = x1;
                    const bool below0 = lane > c, below1 = true;
                    const double l0 = below0 ? (d != 0.0 ? x0 * inv : x0) : x0;
                    const double l1 = (d != 0.0 ? x1 * inv : x1);
#pragma unroll
                    for (int c2 = c + 1; c2 < 8; ++c2) {
                        if (c2 < kb) {
                            const double xj = readlane_d(p0[c], c2);   // unscaled column c at row k0 + c2
                            if (below0 && lane >= c2) p0[c2] -= l0 * xj;
                            if (below1) p1[c2] -= l1 * xj;
                        }
                    }
                    if (below0) p0[c] = l0;
                    p1[c] = l1;
                }
            }
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                if (c < kb) {
                    if (i0 < n && c <= lane) A[i0 * AS + k0 + c] = p0[c];
                    if (i1 < n) A[i1 * AS + k0 + c] = p1[c];
                }
            }
        }
        __syncthreads();
        // trailing update: A[i][j] -= sum_c L[i][c] X[j][c], k0+kb <= j <= i < n, in 4x4 micro-tiles
        const int m0 = k0 + kb;
        const int mt = (n - m0 + 3) >> 2;
        const int ntile = mt * (mt + 1) / 2;
        for (int x = tid; x < ntile; x += CT) {
            int I = (int)((sqrt(8.0 * x + 1.0) - 1.0) * 0.5);
            while ((I + 1) * (I + 2) / 2 <= x) ++I;
            while (I * (I + 1) / 2 > x) --I;
            const int J = x - I * (I + 1) / 2;
            const int rb = m0 + 4 * I, cb = m0 + 4 * J;
            double Lr[4][8], Xc8[4][8];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const int i = rb + r, j = cb + r;
                    Lr[r][c] = (i < n && c < kb) ? A[i * AS + k0 + c] : 0.0;
                    Xc8[r][c] = (j < n && c < kb) ? Xp[j * 8 + c] : 0.0;
                }
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int i = rb + r, j = cb + s;
                    if (i < n && j <= i) {
                        double acc = 0.0;
#pragma unroll
                        for (int c = 0; c < 8; ++c) acc += Lr[r][c] * Xc8[s][c];
                        A[i * AS + j] -= acc;
                    }
                }
        }
        __syncthreads();
    }

    STAMP(12);
    // ---------------- solve: L z = y, z /= D, L^T w = z (LDLT::_solve_impl) ----------------
    if (wave == 0) {
        double z0 = (lane < n) ? yv[lane] : 0.0, z1 = (lane + 64 < n) ? yv[lane + 64] : 0.0;
        for (int k = 0; k < n; ++k) {
            const double zk = (k < 64) ? readlane_d(z0, k) : readlane_d(z1, k - 64);
            if (lane > k && lane < n) z0 -= A[lane * AS + k] * zk;
            if (lane + 64 > k && lane + 64 < n) z1 -= A[(lane + 64) * AS + k] * zk;
        }
        const double tol = 2.2250738585072014e-308;
        if (lane < n) { const double d = Dv[lane]; z0 = fabs(d) > tol ? z0 / d : 0.0; }
        if (lane + 64 < n) { const double d = Dv[lane + 64]; z1 = fabs(d) > tol ? z1 / d : 0.0; }
        for (int k = n - 1; k >= 0; --k) {
            const double zk = (k < 64) ? readlane_d(z0, k) : readlane_d(z1, k - 64);
            if (lane < k) z0 -= A[k * AS + lane] * zk;
            if (lane + 64 < k) z1 -= A[k * AS + lane + 64] * zk;
        }
        if (lane < n) dxp[perm[lane]] = z0;
        if (lane + 64 < n) dxp[perm[lane + 64]] = z1;
    }
    __syncthreads();

    STAMP(13);
    // ---------------- pose part of the gain denominator; candidate poses ----------------
    double sp = 0.0;
    for (int i = tid; i < n; i += CT) {
        const double d = dxp[i];
        const double b = rs[LY.off_bp + i];
        sp += (prm.strategy == 0) ? d * (lambda * d + b) : d * (lambda * rs[LY.off_hd + i] * d + b);
    }
    for (int off = 32; off > 0; off >>= 1) sp += __shfl_xor(sp, off);
    if (lane == 0) s_red[wave] = sp;
    const int cand = 1 - cur;
    if (tid < P) {
        const int pidx = tid;
        double up[6];
        bool bad = false;
        for (int a = 0; a < 6; ++a) { up[a] = dxp[6 * pidx + a]; bad |= !isfinite(up[a]); }
        if (bad) for (int a = 0; a < 6; ++a) up[a] = 0.0;   // VertexPose::add NaN/Inf guard
        // VertexPose::add: estimate_ = (SE3::exp(update) * SE3(estimate_)).matrix()
        double qe[4], te[3], qT[4], qn[4], tr[3], Rn[9];
        d_se3_exp(up, qe, te);
        const double* Tc = pose_mat + ((size_t)cur * P + pidx) * 12;
        const double Rc[9] = {Tc[0], Tc[1], Tc[2], Tc[4], Tc[5], Tc[6], Tc[8], Tc[9], Tc[10]};
        const double tc[3] = {Tc[3], Tc[7], Tc[11]};
        d_q_from_R(Rc, qT);
        d_q_mul(qe, qT, qn);
        d_q_rotate(qe, tc, tr);
        d_R_from_q(qn, Rn);
        double* To = pose_mat + ((size_t)cand * P + pidx) * 12;
        for (int i = 0; i < 3; ++i) {
            To[4 * i] = Rn[3 * i]; To[4 * i + 1] = Rn[3 * i + 1]; To[4 * i + 2] = Rn[3 * i + 2];
            To[4 * i + 3] = te[i] + tr[i];
        }
        for (int cam = 0; cam < prm.ncam; ++cam)
            d_pose_table(To, ext + LH_EXT * cam, ptab + (size_t)cand * P * prm.ncam * LH_PT + (pidx * prm.ncam + cam) * LH_PT);
    }
    __syncthreads();
    if (tid == 0) {
        double s = 0.0;
        for (int w = 0; w < CT / 64; ++w) s += s_red[w];
        ctrl->spose = s;
    }
    STAMP(14);
}

// ============================================================================
// launchers (host side)
// ============================================================================
extern "C" {

hipError_t lh_launch_lin(int T, int trial, int nchunks, int chunk_base, hipStream_t st, const lh_chunk* chunks,
                         const lh_subbatch* sbs, const uint32_t* lm_ptr, const double* obs_uv, const uint32_t* obs_meta,
                         double* Xbuf, double* cache, const double* ptab, const double* ext, const lh_ctrl* ctrl,
                         const double* dxp, double* edge_rho, double* slabs, lh_params prm, int L, uint32_t fixed_mask) {
    if (nchunks <= 0) return hipSuccess;
    dim3 g(nchunks), b(256);
#define LH_LIN(TT, TR) hipLaunchKernelGGL((k_lin<TT, TR>), g, b, 0, st, chunks, sbs, lm_ptr, obs_uv, obs_meta, Xbuf, cache, ptab, ext, ctrl, dxp, edge_rho, slabs, prm, L, fixed_mask, chunk_base)
    switch (T * 2 + (trial ? 1 : 0)) {
        case 2: LH_LIN(1, false); break;
        case 3: LH_LIN(1, true); break;
        case 4: LH_LIN(2, false); break;
        case 5: LH_LIN(2, true); break;
        case 6: LH_LIN(3, false); break;
        case 7: LH_LIN(3, true); break;
        case 8: LH_LIN(4, false); break;
        case 9: LH_LIN(4, true); break;
        default: return hipErrorInvalidValue;
    }
#undef LH_LIN
    return hipGetLastError();
}

hipError_t lh_launch_reduce(hipStream_t st, const lh_chunk* chunks, const double* slabs, const uint32_t* pair_ptr,
                            const uint32_t* items, const uint16_t* pair_pq, const lh_ctrl* ctrl, double* rs_stage,
                            double* maxd, lh_params prm, int n_chunks) {
    (void)chunks;
    const int npairs = prm.P * (prm.P + 1) / 2;
    hipLaunchKernelGGL(k_reduce, dim3(npairs + 1), dim3(RT), 0, st, slabs, pair_ptr, items, pair_pq, ctrl,
                       rs_stage, maxd, prm, n_chunks);
    return hipGetLastError();
}

hipError_t lh_launch_ctrl(hipStream_t st, lh_ctrl* ctrl, double* rs_commit, const double* rs_stage, const double* maxd,
                          double* pose_mat, double* ptab, const double* ext, double* dxp, lh_params prm, int mode,
                          int* host_done) {
    hipLaunchKernelGGL(k_ctrl, dim3(1), dim3(CT), 0, st, ctrl, rs_commit, rs_stage, maxd, pose_mat, ptab, ext, dxp, prm,
                       mode, (volatile int*)host_done);
    return hipGetLastError();
}

// ---- MFMA f64 layout probe (tests): D = A * B for 16x4 A, 4x16 B ----
__global__ void k_mfma_probe(const double* A, const double* B, double* D) {
    const int l = threadIdx.x;
    v4d acc = {0.0, 0.0, 0.0, 0.0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 4 + (l >> 4)], B[(l >> 4) * 16 + (l & 15)], acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) D[((l >> 4) + 4 * i) * 16 + (l & 15)] = acc[i];
}

hipError_t lh_read_stamps(unsigned long long* out, int n, int reset) {
#ifdef LH_STAMPS
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(lh_stamps), sizeof(unsigned long long) * (n < 64 ? n : 64));
    if (e != hipSuccess) return e;
    if (reset) {
        unsigned long long z[64] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(lh_stamps), z, sizeof(z));
    }
    return e;
#else
    for (int i = 0; i < n; ++i) out[i] = 0;
    (void)reset;
    return hipSuccess;
#endif
}

hipError_t lh_launch_mfma_probe(const double* A, const double* B, double* D) {
    hipLaunchKernelGGL(k_mfma_probe, dim3(1), dim3(64), 0, 0, A, B, D);
    return hipGetLastError();
}

}  // extern "C"

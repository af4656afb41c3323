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
#include <algorithm>
#include <math.h>
#include <stdint.h>

#include "lh_common.h"

typedef double v4d __attribute__((ext_vector_type(4)));


// Diagnostic build (-DLH_STAMPS): per-phase wave-cycle totals via s_memtime,
// summed over all waves into lh_stamps[] (cdna_hip_programming.md §7 "In-kernel
// stamps").  The product build compiles these to nothing.
#ifdef LH_STAMPS
__device__ unsigned long long lh_stamps[64];
#define STAMP_DECL unsigned long long st0_ = __builtin_amdgcn_s_memtime(), st1_, sacc_[24] = {0};
#define STAMP(i)                                                                   \
    do {                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                         \
        st1_ = __builtin_amdgcn_s_memtime();                                       \
        sacc_[(i) % 24] += st1_ - st0_;                                            \
        st0_ = st1_;                                                               \
        __builtin_amdgcn_sched_barrier(0);                                         \
    } while (0)
#define STAMP_FLUSH(base, cnt)                                                     \
    do {                                                                           \
        if ((threadIdx.x & 63) == 0)                                               \
            for (int i_ = 0; i_ < (cnt); ++i_)                                     \
                if (sacc_[((base) + i_) % 24]) atomicAdd(&lh_stamps[(base) + i_], sacc_[((base) + i_) % 24]); \
    } while (0)
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_FLUSH(base, cnt)
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
    double w, x, y, z;     // scalars, not an indexed array: keeps the pose code out of scratch
    if (t > 0.0) {
        t = sqrt(t + 1.0);
        w = 0.5 * t;
        t = 0.5 / t;
        x = (R[7] - R[5]) * t;
        y = (R[2] - R[6]) * t;
        z = (R[3] - R[1]) * t;
    } else {
        int i = 0;
        if (R[4] > R[0]) i = 1;
        if (R[8] > (i ? R[4] : R[0])) i = 2;
        // Eigen's c[i], c[j], c[k] with j = (i+1)%3, k = (j+1)%3, written out per case
        if (i == 0) {
            t = sqrt(R[0] - R[4] - R[8] + 1.0);
            x = 0.5 * t; t = 0.5 / t;
            w = (R[7] - R[5]) * t;
            y = (R[3] + R[1]) * t;
            z = (R[6] + R[2]) * t;
        } else if (i == 1) {
            t = sqrt(R[4] - R[8] - R[0] + 1.0);
            y = 0.5 * t; t = 0.5 / t;
            w = (R[2] - R[6]) * t;
            z = (R[7] + R[5]) * t;
            x = (R[1] + R[3]) * t;
        } else {
            t = sqrt(R[8] - R[0] - R[4] + 1.0);
            z = 0.5 * t; t = 0.5 / t;
            w = (R[3] - R[1]) * t;
            x = (R[2] + R[6]) * t;
            y = (R[5] + R[7]) * t;
        }
    }
    q[0] = w; q[1] = x; q[2] = y; q[3] = z;
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
// 1/d with one v_rcp_f64 and two Newton steps (the LDLT pivots and the H_ll Cholesky are not a bitwise-mirrored path)
__device__ __forceinline__ double fast_rcp(double d) {
    double r = __builtin_amdgcn_rcp(d);
    r = fma(r, fma(-d, r, 1.0), r);
    r = fma(r, fma(-d, r, 1.0), r);
    return r;
}

// 1/sqrt(a) with v_rsq_f64 and two Newton steps (the H_ll Cholesky is not a mirrored path)
__device__ __forceinline__ double fast_rsq(double a) {
    double y = __builtin_amdgcn_rsq(a);
    const double h = 0.5 * a;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}

template <int T>
struct LinCfg {
    static constexpr int NT = T * (T + 1) / 2;          // upper MFMA tiles of the window
    static constexpr int GS = (T == 1) ? 16 : (T == 4 ? 80 : 48);  // G row stride: 16T + pad, conflict-free b64 frag loads
    static constexpr int UMAX = (16 * T) / 6;           // window poses that fit 16T rows
    // per-wave LDS scratch: pose-sum image [slot][landmark][33], G image [24][GS], the record
    // stage (128), and (over the 4 waves) the two combine slabs
    static constexpr int A_ = UMAX * LH_SB_LM * LH_TASKS, B_ = 3 * LH_SB_LM * GS, C_ = (2 * LH_SLAB_STRIDE + 3) / 4;
    static constexpr int SCR = ((A_ > B_ ? (A_ > C_ ? A_ : C_) : (B_ > C_ ? B_ : C_)) + 1) & ~1;
};

// butterfly sum over the aligned lane group of G = 1 << lg lanes (every lane gets the total):
// v + v[lane^1], + [lane^2], + [lane^4], ... in that order.  Partners within a 16-lane row come
// through DPP (plain VALU: quad_perm for ^1 and ^2, row rotations for ^4 and ^8); ^16 and ^32
// through ds_bpermute.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(x >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double group_sum(double v, int lg) {
    if (lg >= 1) v += dpp_d<0xB1>(v);                       // quad_perm [1,0,3,2]: lane ^ 1
    if (lg >= 2) v += dpp_d<0x4E>(v);                       // quad_perm [2,3,0,1]: lane ^ 2
    if (lg >= 3) {                                          // lane ^ 4: row_ror 12 / row_ror 4
        const double a = dpp_d<0x12C>(v), b = dpp_d<0x124>(v);
        v += (__lane_id() & 4) ? b : a;
    }
    if (lg >= 4) v += dpp_d<0x128>(v);                      // row_ror 8: lane ^ 8
    if (lg >= 5) v += __shfl_xor(v, 16);
    if (lg >= 6) v += __shfl_xor(v, 32);
    return v;
}

template <int T, bool TRIAL>
__global__ __launch_bounds__(256, (T <= 3) ? 2 : 1) void k_lin(
    const lh_chunk* __restrict__ chunks, const lh_subbatch* __restrict__ sbs, const double* __restrict__ obs_uv,
    const uint32_t* __restrict__ obs_meta, double* __restrict__ rec, const double* __restrict__ pose_tab,
    const double* __restrict__ ext, const lh_ctrl* __restrict__ ctrl, const double* __restrict__ dxp,
    double* __restrict__ edge_rho, double* __restrict__ slabs, lh_params prm, int nrec, uint32_t fixed_mask,
    int chunk_base) {
    using Cfg = LinCfg<T>;
    extern __shared__ __attribute__((aligned(16))) double dsm[];

    if (__builtin_amdgcn_readfirstlane(ctrl->done)) return;
    const int cur = __builtin_amdgcn_readfirstlane(ctrl->cur);
    const int cand = 1 - cur;
    const double lambda = ctrl->lambda;
    const int chunk = chunk_base + blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar loads, scalar loop
    const int ncam = prm.ncam;
    const int PT = prm.P * ncam * LH_PT;
    const int U = chunks[chunk].U;
    const uint32_t sb_begin = chunks[chunk].sb_begin, sb_end = chunks[chunk].sb_end;
    const uint16_t* __restrict__ cpose = chunks[chunk].pose;

    double* scr = dsm + wave * Cfg::SCR;
    // the chunk's window, LDS-resident: committed and candidate pose tables per (slot, camera),
    // the pending pose step per slot, the camera extrinsics
    double* wt_c = dsm + LH_WAVES * Cfg::SCR;
    double* wt_n = wt_c + LH_UMAX * ncam * LH_PT;
    double* wdx = wt_n + LH_UMAX * ncam * LH_PT;
    double* wext = wdx + LH_UMAX * 6;
    {
        const int per = ncam * LH_PT, ne = U * per;
        for (int i = tid; i < ne; i += 256) {
            const int sl = i / per;
            const size_t g = (size_t)cpose[sl] * per + (i - sl * per);
            wt_c[i] = pose_tab[(size_t)cur * PT + g];
            wt_n[i] = pose_tab[(size_t)cand * PT + g];
        }
        if (TRIAL)
            for (int i = tid; i < 6 * U; i += 256) wdx[i] = dxp[6 * cpose[i / 6] + (i - 6 * (i / 6))];
        for (int i = tid; i < ncam * LH_EXT; i += 256) wext[i] = ext[i];
    }

    const double2* __restrict__ rc2 = reinterpret_cast<const double2*>(rec + (size_t)cur * nrec * LH_REC);
    double* __restrict__ rn = rec + (size_t)cand * nrec * LH_REC;

    v4d acc[Cfg::NT];
#pragma unroll
    for (int t = 0; t < Cfg::NT; ++t) acc[t] = v4d{0.0, 0.0, 0.0, 0.0};
    double task[Cfg::UMAX];
#pragma unroll
    for (int u = 0; u < Cfg::UMAX; ++u) task[u] = 0.0;
    double chi_acc = 0.0, scale_acc = 0.0, maxd = 0.0, ndeg = 0.0;
    STAMP_DECL

    // prefetch of the first sub-batch: observation words and the 8 landmark records.  The
    // prefetch is unconditional (index clamped to the chunk) so the compiler can keep it in
    // flight with counted vmcnt waits across the iteration.
    const int sb_last = (int)sb_end - 1;
    int sb = (int)sb_begin + wave;
    uint32_t meta_n;
    double u_n, v_n;
    double2 r_n;
    {
        const int sbc = min(sb, sb_last);
        const int o = sbc * 64 + lane;
        meta_n = obs_meta[o];
        u_n = obs_uv[2 * (size_t)o];
        v_n = obs_uv[2 * (size_t)o + 1];
        r_n = rc2[(size_t)sbc * 64 + lane];
    }
    __syncthreads();   // window tables

    for (; sb < (int)sb_end; sb += LH_WAVES) {
        const lh_subbatch S = sbs[sb];   // scalar load (sb is wave-uniform)
        const int lg = S.lg, nlm = S.n_lm;
        const int ls = lane >> lg, gj = lane & ((1 << lg) - 1);
        const bool lmok = ls < nlm;
        const bool lead = gj == 0 && lmok;           // one lane per landmark writes its record
        const uint32_t meta = meta_n;
        const double u = u_n, v = v_n;
        const double2 rr = r_n;
        const int o = sb * 64 + lane;
        {
            const int sbn = min(sb + LH_WAVES, sb_last);
            const int on = sbn * 64 + lane;
            meta_n = obs_meta[on];
            u_n = obs_uv[2 * (size_t)on];
            v_n = obs_uv[2 * (size_t)on + 1];
            r_n = rc2[(size_t)sbn * 64 + lane];
        }
        // landmark records through LDS: lane -> its landmark's record
        reinterpret_cast<double2*>(scr)[lane] = rr;
        wave_sync();
        const double* myrec = scr + (ls & 7) * LH_REC;
        double X[3] = {myrec[LH_REC_X], myrec[LH_REC_X + 1], myrec[LH_REC_X + 2]};
        double cl[12];
        if (TRIAL) {
#pragma unroll
            for (int i = 0; i < 12; ++i) cl[i] = myrec[LH_REC_L + i];
        }
        wave_sync();

        const bool has = (meta & LH_META_VALID) != 0u;
        const int p = LH_META_POSE(meta), cam = LH_META_CAM(meta), slot = LH_META_SLOT(meta);
        const bool pfixed = (fixed_mask >> p) & 1u;
        const bool live = has && !pfixed;
        const double* e = wext + cam * LH_EXT;
        const bool ext_id = (prm.ext_identity >> cam) & 1;

        // ---- back-substitution of the pending pose step (problem.cpp:426-429) ----
        if (TRIAL) {
            double v3[3] = {0.0, 0.0, 0.0};
            if (live) {
                const double* pt = wt_c + (slot * ncam + cam) * LH_PT;
                EdgeEval E;
                edge_residual(pt, e, ext_id, X, u, v, prm, E.r0, E.r1);
                edge_robust(E, prm);
                edge_jacobians(pt, e, ext_id, X, prm, E.Jp, E.Jl);
                const double* d = wdx + 6 * slot;
                double jd0 = 0.0, jd1 = 0.0;
#pragma unroll
                for (int a = 0; a < 6; ++a) { jd0 += E.Jp[a] * d[a]; jd1 += E.Jp[6 + a] * d[a]; }
                const double y0 = E.W00 * jd0 + E.W01 * jd1, y1 = E.W10 * jd0 + E.W11 * jd1;
#pragma unroll
                for (int c = 0; c < 3; ++c) v3[c] = E.Jl[c] * y0 + E.Jl[3 + c] * y1;
            }
            const double s0 = group_sum(v3[0], lg), s1 = group_sum(v3[1], lg), s2 = group_sum(v3[2], lg);
            if (lmok) {
                // the cached factor holds 1/L_ii on the diagonal
                const double i00 = cl[0], l10 = cl[1], i11 = cl[2], l20 = cl[3], l21 = cl[4], i22 = cl[5];
                const double b0 = cl[6], b1 = cl[7], b2 = cl[8];
                const double t0 = b0 - s0, t1 = b1 - s1, t2 = b2 - s2;
                const double y0 = t0 * i00, y1 = (t1 - l10 * y0) * i11, y2 = (t2 - l20 * y0 - l21 * y1) * i22;
                double d2 = y2 * i22, d1 = (y1 - l21 * d2) * i11, d0 = (y0 - l10 * d1 - l20 * d2) * i00;
                if (prm.guard && !(i00 == i00)) { d0 = d1 = d2 = 0.0; }   // skipped degenerate landmark
                double x0 = X[0], x1 = X[1], x2 = X[2];
                if (isfinite(d0) && isfinite(d1) && isfinite(d2)) { x0 += d0; x1 += d1; x2 += d2; }   // VertexXYZ::add
                if (lead) {
                    double sc;
                    if (prm.strategy == 0) sc = d0 * (lambda * d0 + b0) + d1 * (lambda * d1 + b1) + d2 * (lambda * d2 + b2);
                    else sc = d0 * (lambda * cl[9] * d0 + b0) + d1 * (lambda * cl[10] * d1 + b1) + d2 * (lambda * cl[11] * d2 + b2);
                    scale_acc += sc;
                }
                X[0] = x0; X[1] = x1; X[2] = x2;
            }
        }
        STAMP(0);

        // ---- evaluate and linearise at the candidate (problem.cpp:285-331, :523-526) ----
        // H_pp and b_p go straight to this lane's row of the pose-sum transpose
        double hll[6] = {0, 0, 0, 0, 0, 0}, bl[3] = {0, 0, 0};
        double hpl[18];
#pragma unroll
        for (int i = 0; i < 18; ++i) hpl[i] = 0.0;
        double* trow = scr + (slot * LH_SB_LM + (ls & 7)) * LH_TASKS;   // [slot][landmark][33]: unique writer
        if (has) {
            const double* pt = wt_n + (slot * ncam + cam) * LH_PT;
            EdgeEval E;
            edge_residual(pt, e, ext_id, X, u, v, prm, E.r0, E.r1);
            edge_robust(E, prm);
            edge_jacobians(pt, e, ext_id, X, prm, E.Jp, E.Jl);
            edge_rho[o] = E.rho0;
            chi_acc += E.rho0;
            const double dr = (prm.huber_delta > 0.0) ? E.rho1 : 1.0;
            double WJl[6];
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
                double WJp[12];
#pragma unroll
                for (int a = 0; a < 6; ++a) {
                    WJp[a] = E.W00 * E.Jp[a] + E.W01 * E.Jp[6 + a];
                    WJp[6 + a] = E.W10 * E.Jp[a] + E.W11 * E.Jp[6 + a];
                }
                int k = 0;
#pragma unroll
                for (int a = 0; a < 6; ++a)
#pragma unroll
                    for (int b = a; b < 6; ++b) trow[k++] = E.Jp[a] * WJp[b] + E.Jp[6 + a] * WJp[6 + b];
#pragma unroll
                for (int a = 0; a < 6; ++a) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) hpl[3 * a + c] = E.Jp[a] * WJl[c] + E.Jp[6 + a] * WJl[3 + c];
                    trow[21 + a] = -((dr * E.Jp[a]) * E.r0 + (dr * E.Jp[6 + a]) * E.r1);
                }
            }
        }
        STAMP(1);

        // ---- per-landmark H_ll, b_l over the lane group; Cholesky (redundant per lane) ----
        double h[9];
#pragma unroll
        for (int i = 0; i < 6; ++i) h[i] = group_sum(hll[i], lg);
#pragma unroll
        for (int i = 0; i < 3; ++i) h[6 + i] = group_sum(bl[i], lg);
        // Cholesky of H_ll through reciprocal square roots: i_jj = 1/L_jj directly
        double i00 = fast_rsq(h[0]);
        const double l10 = h[1] * i00, l20 = h[2] * i00;
        const double a11 = h[3] - l10 * l10;
        const double i11 = fast_rsq(a11);
        const double l21 = (h[4] - l20 * l10) * i11;
        const double a22 = h[5] - l20 * l20 - l21 * l21;
        const double i22 = fast_rsq(a22);
        const bool pd = (h[0] > 0.0) && (a11 > 0.0) && (a22 > 0.0) && isfinite(i22) && isfinite(l21);
        if (!pd) i00 = __builtin_nan("");   // poisons the step, like a singular LU inverse (problem.cpp:399)
        const double w0 = h[6] * i00, w1 = (h[7] - l10 * w0) * i11, w2 = (h[8] - l20 * w0 - l21 * w1) * i22;
        if (lead) {
            maxd = fmax(maxd, fmax(fabs(h[0]), fmax(fabs(h[3]), fabs(h[5]))));
            if (!pd) ndeg += 1.0;
            double* rw = rn + ((size_t)sb * LH_SB_LM + ls) * LH_REC;
            reinterpret_cast<double2*>(rw)[0] = double2{X[0], X[1]};
            reinterpret_cast<double2*>(rw)[1] = double2{X[2], i00};
            reinterpret_cast<double2*>(rw)[2] = double2{l10, i11};
            reinterpret_cast<double2*>(rw)[3] = double2{l20, l21};
            reinterpret_cast<double2*>(rw)[4] = double2{i22, h[6]};
            reinterpret_cast<double2*>(rw)[5] = double2{h[7], h[8]};
            reinterpret_cast<double2*>(rw)[6] = double2{h[0], h[3]};
            reinterpret_cast<double2*>(rw)[7] = double2{h[5], 0.0};
        }
        STAMP(2);

        // ---- per observation: G = H_pl L^-T and bsd = G w = H_pl H_ll^-1 b_l ----
        double G[18];
#pragma unroll
        for (int i = 0; i < 18; ++i) G[i] = 0.0;
        const bool gl = live && !(prm.guard && !pd);
        if (gl) {
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                const double g0 = hpl[3 * a] * i00;
                const double g1 = (hpl[3 * a + 1] - l10 * g0) * i11;
                const double g2 = (hpl[3 * a + 2] - l20 * g0 - l21 * g1) * i22;
                G[3 * a] = g0; G[3 * a + 1] = g1; G[3 * a + 2] = g2;
                trow[27 + a] = g0 * w0 + g1 * w1 + g2 * w2;
            }
        } else if (live) {
#pragma unroll
            for (int a = 0; a < 6; ++a) trow[27 + a] = 0.0;
        }
        STAMP(3);

        // ---- per-pose sums (H_pp, b_p, bsd): lane k < 33 adds task k of every landmark observing
        //      the slot, in landmark (= lane) order ----
        wave_sync();
        {
            const int G = 1 << lg;
            const uint64_t gmask = (G == 64) ? ~0ull : ((1ull << G) - 1ull);
#pragma unroll
            for (int uu = 0; uu < Cfg::UMAX; ++uu) {
                if (uu < U) {
                    const uint64_t mk = __ballot(live && slot == uu);
                    if (mk && lane < LH_TASKS) {
                        double tv[LH_SB_LM];
#pragma unroll
                        for (int l = 0; l < LH_SB_LM; ++l) tv[l] = scr[(uu * LH_SB_LM + l) * LH_TASKS + lane];
                        double sacc = task[uu];
#pragma unroll
                        for (int l = 0; l < LH_SB_LM; ++l)
                            if (l < nlm && ((mk >> (l << lg)) & gmask)) sacc += tv[l];
                        task[uu] = sacc;
                    }
                }
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
        if (gl) {
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

    // ---- combine the 4 waves, (w0 + w2) + (w1 + w3), and write the chunk slab ----
    for (int off = 32; off > 0; off >>= 1) {
        chi_acc += __shfl_xor(chi_acc, off);
        scale_acc += __shfl_xor(scale_acc, off);
        ndeg += __shfl_xor(ndeg, off);
        maxd = fmax(maxd, __shfl_xor(maxd, off));
    }
    __syncthreads();
    double* smem = dsm;
    const int ntile = Cfg::NT * 256;
    const int ntask = U * LH_TASKS;
    for (int phase = 0; phase < 2; ++phase) {
        if ((wave >> 1) == phase) {
            double* sl = smem + (wave & 1) * LH_SLAB_STRIDE;
            const bool first = phase == 0;
#pragma unroll
            for (int t = 0; t < Cfg::NT; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int idx = t * 256 + ((lane >> 4) + 4 * i) * 16 + (lane & 15);
                    sl[idx] = (first ? 0.0 : sl[idx]) + acc[t][i];
                }
            if (lane < LH_TASKS) {
#pragma unroll
                for (int uu = 0; uu < Cfg::UMAX; ++uu) {
                    if (uu < U) {
                        const int idx = LH_SLAB_TASK_OFF + uu * LH_TASKS + lane;
                        sl[idx] = (first ? 0.0 : sl[idx]) + task[uu];
                    }
                }
            }
            if (lane == 0) {
                double* sc = sl + LH_SLAB_SC_OFF;
                if (first) { sc[0] = chi_acc; sc[1] = scale_acc; sc[2] = ndeg; sc[3] = maxd; }
                else { sc[0] += chi_acc; sc[1] += scale_acc; sc[2] += ndeg; sc[3] = fmax(sc[3], maxd); }
            }
        }
        __syncthreads();
    }
    const double* s0 = smem;
    const double* s1 = smem + LH_SLAB_STRIDE;
    double* gs = slabs + (size_t)chunk * LH_SLAB_STRIDE;
    for (int i = tid; i < ntile; i += 256) gs[i] = s0[i] + s1[i];
    for (int i = tid; i < ntask; i += 256) gs[LH_SLAB_TASK_OFF + i] = s0[LH_SLAB_TASK_OFF + i] + s1[LH_SLAB_TASK_OFF + i];
    if (tid < 3) gs[LH_SLAB_SC_OFF + tid] = s0[LH_SLAB_SC_OFF + tid] + s1[LH_SLAB_SC_OFF + tid];
    if (tid == 3) gs[LH_SLAB_SC_OFF + 3] = fmax(s0[LH_SLAB_SC_OFF + 3], s1[LH_SLAB_SC_OFF + 3]);
    STAMP(7);
    STAMP_FLUSH(0, 8);
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
#define RI_MAX 2048           // items (chunks) per pose pair staged in LDS at a time

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
    int off_h = 0;
    if (lane < 36) off_h = LH_SLAB_TASK_OFF + (diag ? ((a < bb ? a : bb) * 6 - ((a < bb ? a : bb) * ((a < bb ? a : bb) - 1)) / 2 + ((a < bb ? bb : a) - (a < bb ? a : bb))) : 0);
    else if (lane < 42) off_h = LH_SLAB_TASK_OFF + 21 + (lane - 36);
    else if (lane < 48) off_h = LH_SLAB_TASK_OFF + 27 + (lane - 42);
    const bool act_s = lane < 36, act_h = (lane < 36 && diag) || (lane >= 36 && lane < 48 && diag);
    __shared__ uint32_t sitems[RI_MAX];
    auto slab_off = [&](uint32_t item, int& off_s, const double*& sl) {
        const int ch = item >> 11, T = (item >> 8) & 7, sp = (item >> 4) & 15, sq = item & 15;
        sl = slabs + (size_t)ch * LH_SLAB_STRIDE;
        int ra = 6 * sp + a, rc = 6 * sq + bb;
        if ((ra >> 4) > (rc >> 4)) { const int t = ra; ra = rc; rc = t; }
        const int R = ra >> 4, Cc = rc >> 4;
        off_s = act_s ? (R * T - (R * (R - 1)) / 2 + (Cc - R)) * 256 + (ra & 15) * 16 + (rc & 15) : 0;
        return sp;
    };
    double vs = 0.0, vh = 0.0;
    const int ib = pair_ptr[b], ie = pair_ptr[b + 1];
    for (int seg = ib; seg < ie; seg += RI_MAX) {
        // a segment of the pair's item list into LDS (one global round trip), then every wave
        // walks its items (wave, wave + RW, ...) with four slab loads in flight
        const int nit = min(ie - seg, RI_MAX);
        __syncthreads();
        for (int i = tid; i < nit; i += RT) sitems[i] = items[seg + i];
        __syncthreads();
        int it = wave;
        for (; it + 3 * RW < nit; it += 4 * RW) {
            double x[4], y[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                int off_s; const double* sl;
                const int sp = slab_off(sitems[it + u * RW], off_s, sl);
                x[u] = act_s ? sl[off_s] : 0.0;
                y[u] = act_h ? sl[off_h + sp * LH_TASKS] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) { vs += x[u]; vh += y[u]; }
        }
        for (; it < nit; it += RW) {
            int off_s; const double* sl;
            const int sp = slab_off(sitems[it], off_s, sl);
            if (act_s) vs += sl[off_s];
            if (act_h) vh += sl[off_h + sp * LH_TASKS];
        }
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
    STAMP_FLUSH(20, 1);
}

// ============================================================================
// k_ctrl: LM controller + reduced-system solve, one workgroup of 256 threads.
//
//  1. one global round trip: every thread prefetches its slice of BOTH reduced
//     systems (staged candidate linearisation and committed one) plus the
//     controller and pose matrices, while thread 0 runs isGoodStepInLM;
//  2. the chosen system is scattered straight from registers into LDS in Eigen's
//     LDLT pivot order (problem.cpp:420; left-looking Eigen LDLT pivots on the
//     ORIGINAL |diag|, so the order is a static sort), committing it on accept;
//  3. right-looking blocked LDL^T, panel 8: every panel thread factors the 8x8
//     diagonal block redundantly in registers (no cross-lane chain), then its
//     own row; the right-hand side rides along as an extra row (row NP), so the
//     forward substitution is part of the factorisation;
//  4. blocked back substitution in one wave; candidate poses (VertexPose::add).
// The matrix is padded to NE = ceil8(n) with identity rows: no bounds tests in
// the inner loops.
// ============================================================================
#define CT 512
#define NP LH_NPAD            // padded system size; row NP of A holds the right-hand side
#define AS (LH_NPAD + 1)      // LDS row stride (odd: row-per-lane access is conflict-free)
#define XS 9                  // LDS row stride of the panel's unscaled columns
#define RS_MAX (LH_PMAX * (LH_PMAX + 1) / 2 * 36 + 18 * LH_PMAX + 8)
#define NLD ((RS_MAX + CT - 1) / CT)


#define TRI8(r, c) ((r) * ((r) - 1) / 2 + (c))   // packed strictly-lower 8x8 index, r > c

// LDL^T of the 8x8 diagonal block at (k0, k0) of A (lower triangle), computed redundantly by
// every lane of one wave; one lane writes D on A's diagonal and L below it (L = W where Eigen's
// pivot_is_valid fails, ldlt_inplace).  Stores from one wave are slow: only these 36 values.
__device__ __forceinline__ void factor_block8(double* A, int k0, int lane) {
    double B[8][8], Wb[8][8], dv[8], inv[8];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int c = 0; c <= r; ++c) B[r][c] = A[(k0 + r) * AS + k0 + c];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        dv[c] = B[c][c];
        const bool valid = fabs(dv[c]) > 0.0;     // Eigen ldlt_inplace: pivot_is_valid
        inv[c] = valid ? fast_rcp(dv[c]) : 1.0;
#pragma unroll
        for (int r = c + 1; r < 8; ++r) Wb[r][c] = B[r][c];
#pragma unroll
        for (int r = c + 1; r < 8; ++r) {
            const double l = Wb[r][c] * inv[c];
            B[r][c] = l;
#pragma unroll
            for (int r2 = c + 1; r2 <= r; ++r2) B[r][r2] -= l * Wb[r2][c];
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
#pragma unroll
            for (int c = 0; c < r; ++c) A[(k0 + r) * AS + k0 + c] = B[r][c];
            A[(k0 + r) * AS + k0 + r] = dv[r];
        }
    }
}

// lower-triangular 16x16 tile enumeration x -> (I, J), x = I (I + 1) / 2 + J, I < 8
__constant__ unsigned char c_triI[36] = {0, 1, 1, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 4, 5, 5, 5, 5, 5, 5,
                                         6, 6, 6, 6, 6, 6, 6, 7, 7, 7, 7, 7, 7, 7, 7};
__constant__ unsigned char c_triJ[36] = {0, 0, 1, 0, 1, 2, 0, 1, 2, 3, 0, 1, 2, 3, 4, 0, 1, 2, 3, 4, 5,
                                         0, 1, 2, 3, 4, 5, 6, 0, 1, 2, 3, 4, 5, 6, 7};

// Phases 3-4 of k_ctrl on a permuted, padded system already in LDS (A lower + rhs row NP):
// blocked LDL^T and the solve; xsol[r] = solution in pivot order for r < n.  Shared with the
// k_ldlt_probe test hook.  Must be called by all CT threads.
__device__ __forceinline__ void lds_ldlt_solve(double* __restrict__ A, double* __restrict__ Xp, double* __restrict__ xsol,
                                               int n, int NE, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
#ifdef LH_STAMPS
    unsigned long long st0_ = __builtin_amdgcn_s_memtime(), st1_, sacc_[24] = {0};
#endif
    // ---------------- 3. blocked right-looking LDL^T (+ forward substitution in row NP) ----------------
    // Each 8x8 diagonal block is factored by wave 0 as soon as the previous trailing update has
    // produced it (look-ahead), while the other waves finish that update; the panel phase then
    // only solves every row below against the factored block.
    if (wave == 0) factor_block8(A, 0, lane);
    __syncthreads();
    STAMP(18);
    for (int k0 = 0; k0 < NE; k0 += 8) {
        const int m0 = k0 + 8;
        const int nrow = NE - m0 + 1;                 // panel rows k0+8..NE-1 and the rhs row
        if (tid < nrow) {
            const int i = (tid == nrow - 1) ? NP : m0 + tid;
            // the factored diagonal block: 1/D and W = L D (L itself where the pivot is invalid)
            double inv[8], Wb[28], a[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const double d = A[(k0 + c) * AS + k0 + c];
                const bool valid = fabs(d) > 0.0;
                inv[c] = valid ? fast_rcp(d) : 1.0;
#pragma unroll
                for (int r = c + 1; r < 8; ++r) {
                    const double l = A[(k0 + r) * AS + k0 + c];
                    Wb[TRI8(r, c)] = valid ? l * d : l;
                }
            }
#pragma unroll
            for (int c = 0; c < 8; ++c) a[c] = A[i * AS + k0 + c];
            double w[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                w[c] = a[c];
                const double l = a[c] * inv[c];
                a[c] = l;
#pragma unroll
                for (int c2 = c + 1; c2 < 8; ++c2) a[c2] -= l * Wb[TRI8(c2, c)];
            }
#pragma unroll
            for (int c = 0; c < 8; ++c) A[i * AS + k0 + c] = a[c];
            if (i < NP) {
#pragma unroll
                for (int c = 0; c < 8; ++c) Xp[i * XS + c] = w[c];
            }
        }
        __syncthreads();
        STAMP(15);
        if (m0 < NE) {
            // trailing update A[i][j] -= sum_c L[i][c] W[j][c], k0+8 <= j <= i < NE, on f64 MFMA:
            // 16x16 tiles anchored at tb = floor16(k0+8), two 16x16x4 steps each; rows/cols
            // below k0+8 of the first tile row/col are the panel's own L and D (written back unchanged).
            // Tile 0 holds the next diagonal block: wave 0 updates it first, then factors the block.
            const int tb = m0 & ~15;
            const int mt = (NE - tb) >> 4;
            const int ntile = mt * (mt + 1) / 2;
            const int wv = __builtin_amdgcn_readfirstlane(wave);
            const int li = lane & 15, lk = lane >> 4;
            // wave 4 shares wave 0's SIMD (waves w and w+4 of a workgroup do): it stays idle so the
            // factor chain issues unimpeded; waves 1-3, 5-7 take tiles 1.. round-robin
            const int tq = wv - 1 - (wv > 4 ? 1 : 0);
            const int x0 = (wv == 0) ? 0 : (wv == 4 ? ntile : 1 + tq);
            const int xs_ = (wv == 0) ? ntile : 6;
            for (int x = x0; x < ntile; x += xs_) {
                const int rb = tb + 16 * c_triI[x], cb = tb + 16 * c_triJ[x];
                const double a0 = A[(rb + li) * AS + k0 + lk], a1 = A[(rb + li) * AS + k0 + 4 + lk];
                const double b0 = Xp[(cb + li) * XS + lk], b1 = Xp[(cb + li) * XS + 4 + lk];
                const int col = cb + li;
                double old[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) old[r] = A[(rb + lk + 4 * r) * AS + col];
                v4d acc = {0.0, 0.0, 0.0, 0.0};
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = rb + lk + 4 * r;
                    A[row * AS + col] = (row >= m0 && col >= m0) ? old[r] - acc[r] : old[r];
                }
            }
            if (wv == 0) { STAMP(22); } else { STAMP(23); }
            if (wv == 0) {
                wave_sync();
                factor_block8(A, m0, lane);
                STAMP(12);
            }
            if (tid >= CT - 64) {   // the rhs row (forward substitution): last wave, after its tiles
                for (int j = m0 + (tid - (CT - 64)); j < NE; j += 64) {
                    double acc = 0.0;
#pragma unroll
                    for (int c = 0; c < 8; ++c) acc += A[NP * AS + k0 + c] * Xp[j * XS + c];
                    A[NP * AS + j] -= acc;
                }
            }
            __syncthreads();
        }
        STAMP(16);
    }

    // ---------------- 4. z /= D (Eigen tolerance), back substitution L^T x = z ----------------
    // One wave; the right-hand side lives in LDS (xsol), block rows are read as broadcasts:
    // no readlane chains (2.4x faster than a register-resident rhs, tools/ubench_backsub.hip).
    if (wave == 0) {
        const double tol = 2.2250738585072014e-308;   // LDLT::_solve_impl: (numeric_limits::min)()
        const int r0 = lane, r1 = lane + 64, r1m = r1 & (NP - 1);
        if (r0 < NE) { const double d = A[r0 * AS + r0]; xsol[r0] = fabs(d) > tol ? A[NP * AS + r0] : 0.0; }
        if (r1 < NE) { const double d = A[r1 * AS + r1]; xsol[r1] = fabs(d) > tol ? A[NP * AS + r1] : 0.0; }
        wave_sync();
        for (int kb = NE - 8; kb >= 0; kb -= 8) {
            double Lb[28], x[8], c0[8], c1[8];
#pragma unroll
            for (int w2 = 1; w2 < 8; ++w2)
#pragma unroll
                for (int v = 0; v < w2; ++v) Lb[TRI8(w2, v)] = A[(kb + w2) * AS + kb + v];
#pragma unroll
            for (int v = 0; v < 8; ++v) { c0[v] = A[(kb + v) * AS + r0]; c1[v] = A[(kb + v) * AS + r1m]; }
#pragma unroll
            for (int v = 0; v < 8; ++v) x[v] = xsol[kb + v];
#pragma unroll
            for (int v = 7; v >= 0; --v)
#pragma unroll
                for (int w2 = v + 1; w2 < 8; ++w2) x[v] -= Lb[TRI8(w2, v)] * x[w2];
            double s0 = 0.0, s1 = 0.0;
#pragma unroll
            for (int v = 0; v < 8; ++v) { s0 += c0[v] * x[v]; s1 += c1[v] * x[v]; }
            if (lane == 0) {   // the block's solution: four 16-B stores from one lane (NaN-safe, no selects)
                double2* xb = reinterpret_cast<double2*>(xsol + kb);
                xb[0] = double2{x[0], x[1]}; xb[1] = double2{x[2], x[3]};
                xb[2] = double2{x[4], x[5]}; xb[3] = double2{x[6], x[7]};
            }
            if (r0 < kb) xsol[r0] -= s0;
            if (r1 < kb) xsol[r1] -= s1;
            wave_sync();
        }
    }
    __syncthreads();
    STAMP(13);

#ifdef LH_STAMPS
    STAMP_FLUSH(10, 14);
#endif
}

__global__ __launch_bounds__(CT) void k_ctrl(lh_ctrl* __restrict__ ctrl, double* __restrict__ rs_commit,
                                             const double* __restrict__ rs_stage, const double* __restrict__ maxd_in,
                                             const uint32_t* __restrict__ rsmap,
                                             double* __restrict__ pose_mat, double* __restrict__ ptab,
                                             const double* __restrict__ ext, double* __restrict__ dxp, lh_params prm,
                                             int mode /* 0 init, 1 trial */, volatile int* __restrict__ host_done) {
    __shared__ double A[(NP + 1) * AS];   // permuted S + lambda D (lower); L and D in place; row NP = rhs -> z / D
    __shared__ double Xp[NP * XS];        // unscaled panel columns (W = L D) for the trailing update
    __shared__ double dg[NP], bsv[NP], bpv[NP], hdv[NP], xs[NP];
    __shared__ __attribute__((aligned(16))) double yv[NP];
    __shared__ int perm[NP], iperm[NP];
    __shared__ int s_flags[4];
    __shared__ double s_red[CT / 64], s_lam;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int P = prm.P, n = 6 * P, NE = (n + 15) & ~15;
    const lh_rs_layout LY = lh_rs_make(P);
    STAMP_DECL

    // ---------------- 1. prefetch (one round trip); the controller's words first ----------------
    double chi = 0.0, lam = 0.0, ni = 0.0, last = 0.0, spose = 0.0, chi0 = 0.0, tchi = 0.0, sl = 0.0;
    int iter = 0, fc = 0, trials = 0, nacc = 0, done0 = 1, cur0 = 0, tl = 0;
    if (tid == 0) {
        chi = ctrl->chi; lam = ctrl->lambda; ni = ctrl->ni; last = ctrl->last_chi; spose = ctrl->spose;
        chi0 = ctrl->chi2_initial;
        iter = ctrl->iter; fc = ctrl->false_cnt; trials = ctrl->trials; nacc = ctrl->accepted;
        done0 = ctrl->done; cur0 = ctrl->cur; tl = ctrl->trace_len;
        tchi = 0.5 * rs_stage[LY.off_sc + LH_SC_CHI2];
        sl = rs_stage[LY.off_sc + LH_SC_SCALE];
    }
    double vs[NLD], vc[NLD];
    uint32_t mp[NLD];
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
        const int i = u * CT + tid;
        const bool in = i < LY.total;
        vs[u] = in ? rs_stage[i] : 0.0;
        vc[u] = in ? rs_commit[i] : 0.0;
        mp[u] = i < LY.off_bs ? rsmap[i] : 0u;
    }
    double pm0[12], pm1[12];
    if (tid < P) {
#pragma unroll
        for (int i = 0; i < 12; ++i) { pm0[i] = pose_mat[(size_t)tid * 12 + i]; pm1[i] = pose_mat[((size_t)P + tid) * 12 + i]; }
    }
    if (mode == 0) {   // max |diag H_pp| for computeLambdaInitLM (problem.cpp:486-496)
        double mx = 0.0;
#pragma unroll
        for (int u = 0; u < NLD; ++u) {
            const int i = u * CT + tid;
            if (i >= LY.off_hd && i < LY.off_hd + n) mx = fmax(mx, fabs(vs[u]));
        }
        for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
        if (lane == 0) s_red[wave] = mx;
        __syncthreads();
    }

    // ---------------- LM bookkeeping (thread 0) ----------------
    if (tid == 0) {
        int done = done0, cur = cur0;
        int accept = 0, trace = 0;
        if (!done) {
            if (mode == 0) {
                // computeLambdaInitLM (problem.cpp:470-504)
                ni = 2.0;
                chi = tchi;
                chi0 = tchi;
                if (prm.strategy == 0) {
                    if (!prm.lambda_given) {
                        double m = 0.0;
                        for (int w = 0; w < CT / 64; ++w) m = fmax(m, s_red[w]);
                        m = fmax(*maxd_in, m);
                        m = fmin(prm.lambda_cap, m);
                        lam = prm.tau * m;
                    } else {
                        lam = prm.lambda_init;
                    }
                } else {
                    lam = 1e-5;
                }
                last = 1e20;
                iter = 0; fc = 0; trials = 0; nacc = 0; tl = 0;
                cur = 1 - cur;           // the initial linearisation becomes the committed one
                accept = 1;
                if (prm.max_iters <= 0) done = 1;
                else trace = 1;
            } else {
                // isGoodStepInLM (problem.cpp:520-581)
                double scale = 0.5 * (spose + sl);
                scale += 1e-10;
                const double rho = (chi - tchi) / scale;
                const bool ok = rho > 0 && isfinite(tchi);
                if (prm.strategy == 0) {
                    if (ok) {
                        double alpha = 1.0 - pow((2 * rho - 1), 3);
                        alpha = fmin(alpha, 2.0 / 3.0);
                        lam *= fmax(1.0 / 3.0, alpha);
                        ni = 2;
                        chi = tchi;
                    } else {
                        lam *= ni;
                        ni *= 2;
                    }
                } else {
                    if (ok) { lam = fmax(lam / 9.0, 1e-7); chi = tchi; }
                    else lam = fmin(lam * 11.0, 1e7);
                }
                trials += 1;
                bool inner_end;
                if (ok) {
                    nacc += 1;
                    cur = 1 - cur;       // commit candidate landmarks, caches and poses
                    accept = 1;
                    fc = 0;
                    inner_end = true;
                } else {
                    fc += 1;             // rollbackStates: the committed buffers are untouched
                    inner_end = fc >= prm.max_trials;
                }
                if (inner_end) {
                    iter += 1;
                    if (last - chi < prm.stop_dchi2) done = 1;
                    last = chi;
                    if (!done && iter >= prm.max_iters) done = 1;
                    if (!done) { fc = 0; trace = 1; }
                }
            }
            if (trace) {
                if (tl < LH_TRACE) { ctrl->trace_chi[tl] = chi; ctrl->trace_lambda[tl] = lam; }
                tl += 1;
            }
            ctrl->chi = chi; ctrl->lambda = lam; ctrl->ni = ni; ctrl->last_chi = last; ctrl->chi2_initial = chi0;
            ctrl->iter = iter; ctrl->false_cnt = fc; ctrl->trials = trials; ctrl->accepted = nacc;
            ctrl->done = done; ctrl->cur = cur; ctrl->trace_len = tl;
            if (done && host_done) *host_done = 1;
        }
        s_flags[0] = done;
        s_flags[1] = accept;
        s_flags[2] = cur;
        s_lam = lam;
    }
    __syncthreads();
    const int done = s_flags[0], accept = s_flags[1], cur = s_flags[2];
    if (done) return;
    const double lambda = s_lam;
    STAMP(17);

    // ---------------- 2. commit, diag + lambda, pivot order, scatter into LDS ----------------
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
        const int i = u * CT + tid;
        const double v = accept ? vs[u] : vc[u];
        vs[u] = v;
        if (accept && i < LY.total) rs_commit[i] = v;
        if (i < LY.off_bs) {
            const int gi = mp[u] & 0xff, gj = (mp[u] >> 8) & 0xff;
            if (gi == gj) dg[gi] = (prm.strategy == 0) ? v + lambda : v + lambda * v;
        } else if (i < LY.off_bp) {
            bsv[i - LY.off_bs] = v;
        } else if (i < LY.off_hd) {
            bpv[i - LY.off_bp] = v;
        } else if (i < LY.off_hd + n) {
            hdv[i - LY.off_hd] = v;
        }
    }
    if (tid >= n && tid < NP) dg[tid] = __builtin_nan("");   // key -1 at an index above every real row: never counted
    __syncthreads();
    STAMP(19);
    {
        // |diag| descending; total order (NaN last, ties by index) keeps perm a permutation.
        // Four threads per row, each counting over 32 of the 128 keys (dg[n..NP) are NaN).
        const int row = tid >> 2, part = tid & 3;
        int r = 0;
        if (row < n) {
            double di = fabs(dg[row]);
            if (!(di == di)) di = -1.0;
#pragma unroll
            for (int j0 = 0; j0 < 32; j0 += 8) {
                double dj[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) dj[u] = dg[part * 32 + j0 + u];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    double d = fabs(dj[u]);
                    if (!(d == d)) d = -1.0;
                    r += (d > di) || (d == di && part * 32 + j0 + u < row);
                }
            }
        }
        r += __shfl_xor(r, 1);
        r += __shfl_xor(r, 2);
        if (part == 0 && row < NP) {
            const int rr = row < n ? r : row;
            perm[rr] = row;
            iperm[row] = rr;
        }
    }
    __syncthreads();
    STAMP(21);
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
        const int i = u * CT + tid;
        if (i < LY.off_bs) {
            const int ri = iperm[mp[u] & 0xff], rj = iperm[(mp[u] >> 8) & 0xff];
            if (!(mp[u] >> 16)) A[max(ri, rj) * AS + min(ri, rj)] = vs[u];
            else if (ri > rj) A[ri * AS + rj] = vs[u];
        }
    }
    if (tid < NE) {
        A[tid * AS + tid] = tid < n ? dg[perm[tid]] : 1.0;
        A[NP * AS + tid] = tid < n ? bsv[perm[tid]] : 0.0;
    }
    for (int x = tid; x < (NE - n) * NE; x += CT) {   // identity padding rows
        const int r = n + x / NE, c = x - NE * (x / NE);
        if (c < r) A[r * AS + c] = 0.0;
    }
    __syncthreads();
    STAMP(11);

    // ---------------- 3-4. blocked LDL^T with the forward substitution in row NP; back substitution ----------------
    STAMP_FLUSH(10, 14);
    lds_ldlt_solve(A, Xp, yv, n, NE, tid);
    if (tid < n) { xs[perm[tid]] = yv[tid]; dxp[perm[tid]] = yv[tid]; }
    __syncthreads();
#ifdef LH_STAMPS
    st0_ = __builtin_amdgcn_s_memtime();
    for (int i_ = 0; i_ < 24; ++i_) sacc_[i_] = 0;
#endif
    STAMP(10);

    // ---------------- pose part of the gain denominator; candidate poses ----------------
    double sp = 0.0;
    if (tid < n) {
        const double d = xs[tid], b = bpv[tid];
        sp = (prm.strategy == 0) ? d * (lambda * d + b) : d * (lambda * hdv[tid] * d + b);
    }
    for (int off = 32; off > 0; off >>= 1) sp += __shfl_xor(sp, off);
    if (lane == 0) s_red[wave] = sp;
    const int cand = 1 - cur;
    if (tid < P) {
        const int pidx = tid;
        double up[6];
        bool bad = false;
#pragma unroll
        for (int a = 0; a < 6; ++a) { up[a] = xs[6 * pidx + a]; bad |= !isfinite(up[a]); }
        if (bad) {
#pragma unroll
            for (int a = 0; a < 6; ++a) up[a] = 0.0;   // VertexPose::add NaN/Inf guard
        }
        // VertexPose::add: estimate_ = (SE3::exp(update) * SE3(estimate_)).matrix()
        double qe[4], te[3], qT[4], qn[4], tr[3], Rn[9];
        d_se3_exp(up, qe, te);
        double Tc[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) Tc[i] = cur ? pm1[i] : pm0[i];
        const double Rc[9] = {Tc[0], Tc[1], Tc[2], Tc[4], Tc[5], Tc[6], Tc[8], Tc[9], Tc[10]};
        const double tc[3] = {Tc[3], Tc[7], Tc[11]};
        d_q_from_R(Rc, qT);
        d_q_mul(qe, qT, qn);
        d_q_rotate(qe, tc, tr);
        d_R_from_q(qn, Rn);
        double To[12];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            To[4 * i] = Rn[3 * i]; To[4 * i + 1] = Rn[3 * i + 1]; To[4 * i + 2] = Rn[3 * i + 2];
            To[4 * i + 3] = te[i] + tr[i];
        }
        double* Tg = pose_mat + ((size_t)cand * P + pidx) * 12;
#pragma unroll
        for (int i = 0; i < 12; ++i) Tg[i] = To[i];
        for (int cam = 0; cam < prm.ncam; ++cam)
            d_pose_table(To, ext + LH_EXT * cam, ptab + (size_t)cand * P * prm.ncam * LH_PT + (pidx * prm.ncam + cam) * LH_PT);
    }
    __syncthreads();
    if (tid == 0) {
        double s2 = 0.0;
        for (int w = 0; w < CT / 64; ++w) s2 += s_red[w];
        ctrl->spose = s2;
    }
    STAMP(14);
    STAMP_FLUSH(10, 14);
}

// ============================================================================
// launchers (host side)
// ============================================================================
extern "C" {

static size_t lin_smem_bytes(int scr, int ncam) {
    return sizeof(double) * ((size_t)LH_WAVES * scr + 2 * (size_t)LH_UMAX * ncam * LH_PT + LH_UMAX * 6 + (size_t)ncam * LH_EXT);
}

// Raise the dynamic-LDS limit of every k_lin instantiation on the current device (lh_create), before any
// launch or stream capture.
hipError_t lh_prepare_lin() {
    {
        const void* fns[] = {reinterpret_cast<const void*>(&k_lin<1, false>), reinterpret_cast<const void*>(&k_lin<1, true>),
                             reinterpret_cast<const void*>(&k_lin<2, false>), reinterpret_cast<const void*>(&k_lin<2, true>),
                             reinterpret_cast<const void*>(&k_lin<3, false>), reinterpret_cast<const void*>(&k_lin<3, true>),
                             reinterpret_cast<const void*>(&k_lin<4, false>), reinterpret_cast<const void*>(&k_lin<4, true>)};
        for (const void* f : fns) {
            hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
}

hipError_t lh_launch_lin(int T, int trial, int nchunks, int chunk_base, hipStream_t st, const lh_chunk* chunks,
                         const lh_subbatch* sbs, const double* obs_uv, const uint32_t* obs_meta, double* rec,
                         const double* ptab, const double* ext, const lh_ctrl* ctrl, const double* dxp,
                         double* edge_rho, double* slabs, lh_params prm, int nrec, uint32_t fixed_mask) {
    if (nchunks <= 0) return hipSuccess;
    dim3 g(nchunks), b(256);
#define LH_LIN(TT, TR)                                                                                             \
    do {                                                                                                           \
        const size_t smem = lin_smem_bytes(LinCfg<TT>::SCR, prm.ncam);                                 \
        hipLaunchKernelGGL((k_lin<TT, TR>), g, b, smem, st, chunks, sbs, obs_uv, obs_meta, rec, ptab, ext, ctrl, dxp, \
                           edge_rho, slabs, prm, nrec, fixed_mask, chunk_base);                                    \
    } while (0)
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
                          const uint32_t* rsmap, double* pose_mat, double* ptab, const double* ext, double* dxp, lh_params prm, int mode,
                          int* host_done) {
    hipLaunchKernelGGL(k_ctrl, dim3(1), dim3(CT), 0, st, ctrl, rs_commit, rs_stage, maxd, rsmap, pose_mat, ptab, ext, dxp, prm,
                       mode, (volatile int*)host_done);
    return hipGetLastError();
}

// ---- k_reset: restart a resident solve (one launch instead of five copies) ----
__global__ __launch_bounds__(256) void k_reset(double2* __restrict__ rec, const double2* __restrict__ rec_init, long nrec2,
                                               double* __restrict__ qt, const double* __restrict__ qt_init, int nqt,
                                               double* __restrict__ ptab, const double* __restrict__ ptab_init, int nptab,
                                               double* __restrict__ dxp, int ndxp, lh_ctrl* __restrict__ ctrl) {
    const long i0 = (long)blockIdx.x * 256 + threadIdx.x, st = (long)gridDim.x * 256;
    for (long i = i0; i < nrec2; i += st) rec[i] = rec_init[i];
    if (blockIdx.x == 0) {
        for (int i = threadIdx.x; i < nqt; i += 256) qt[i] = qt_init[i];
        for (int i = threadIdx.x; i < nptab; i += 256) ptab[i] = ptab_init[i];
        for (int i = threadIdx.x; i < ndxp; i += 256) dxp[i] = 0.0;
        int* c = reinterpret_cast<int*>(ctrl);
        for (int i = threadIdx.x; i < (int)(sizeof(lh_ctrl) / sizeof(int)); i += 256) c[i] = 0;   // cur = 0
    }
}

hipError_t lh_launch_reset(hipStream_t st, double* rec, const double* rec_init, long nrec_doubles, double* qt,
                           const double* qt_init, int nqt, double* ptab, const double* ptab_init, int nptab, double* dxp,
                           int ndxp, lh_ctrl* ctrl) {
    const long n2 = nrec_doubles / 2;
    const int blocks = (int)std::max(1L, std::min(2048L, (n2 + 255) / 256));
    hipLaunchKernelGGL(k_reset, dim3(blocks), dim3(256), 0, st, reinterpret_cast<double2*>(rec),
                       reinterpret_cast<const double2*>(rec_init), n2, qt, qt_init, nqt, ptab, ptab_init, nptab, dxp,
                       ndxp, ctrl);
    return hipGetLastError();
}

// ---- LDL^T probe (tests): x = (S)^-1 b through k_ctrl's pivot order, LDS layout and
//      lds_ldlt_solve, for a dense symmetric S (row-major n x n, n <= LH_NPAD) ----
__global__ __launch_bounds__(CT) void k_ldlt_probe(const double* __restrict__ S, const double* __restrict__ b, int n,
                                                   double* __restrict__ x) {
    __shared__ double A[(NP + 1) * AS];
    __shared__ double Xp[NP * XS];
    __shared__ double dg[NP];
    __shared__ __attribute__((aligned(16))) double xsol[NP];
    __shared__ int perm[NP];
    const int tid = threadIdx.x, NE = (n + 15) & ~15;
    if (tid < NP) dg[tid] = tid < n ? S[(size_t)tid * n + tid] : __builtin_nan("");
    __syncthreads();
    if (tid < n) {
        double di = fabs(dg[tid]);
        if (!(di == di)) di = -1.0;
        int r = 0;
        for (int j = 0; j < NP; ++j) {
            double d = fabs(dg[j]);
            if (!(d == d)) d = -1.0;
            r += (d > di) || (d == di && j < tid);
        }
        perm[r] = tid;
    } else if (tid < NP) {
        perm[tid] = tid;
    }
    __syncthreads();
    for (int e = tid; e < NE * NE; e += CT) {
        const int r = e / NE, c = e - NE * (e / NE);
        if (c <= r) A[r * AS + c] = (r < n) ? ((c < n) ? S[(size_t)perm[r] * n + perm[c]] : 0.0) : (r == c ? 1.0 : 0.0);
    }
    if (tid < NE) A[NP * AS + tid] = tid < n ? b[perm[tid]] : 0.0;
    __syncthreads();
    lds_ldlt_solve(A, Xp, xsol, n, NE, tid);
    __syncthreads();
    if (tid < n) x[perm[tid]] = xsol[tid];
}

hipError_t lh_launch_ldlt_probe(const double* S, const double* b, int n, double* x) {
    if (n < 1 || n > LH_NPAD) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ldlt_probe, dim3(1), dim3(CT), 0, 0, S, b, n, x);
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

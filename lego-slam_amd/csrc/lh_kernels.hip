// lh_kernels.hip — CDNA4 (gfx950) kernels of the sliding-window BA solver.
//
// One LM trial of lego::Problem::solve (src/lego/base/problem.cpp:179-220) is
//   k_lin     landmark chunks: back-substitute the pending pose step into the
//             landmarks, evaluate chi2 at the candidate state and relinearise
//             there (residual, SE(3)/point Jacobians, Huber weights, H_pp, H_pl,
//             H_ll, b), eliminate the landmarks (Schur) — the landmark part as
//             an f64 MFMA SYRK over a chunk window — and emit one slab per chunk.
//   k_reduce  fixed-order sum of the pair rows into the reduced pose system.
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
__device__ unsigned long long lh_stamps[256];   // [64, 128): k_ctrl's LDL^T steps, per step (lds_ldlt_solve);
                                                // [128, 160): k_ctrl_b's barrier arrival per wave, even / odd steps
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
// k_ctrl wall-clock stamps: thread 0 (wave 0, the critical chain) adds s_memtime at each
// barrier-aligned phase boundary of every live launch into lh_stamps[32 + i]; consecutive sums
// difference to per-phase latency.  [61] live launches, [62]/[63] s_memrealtime at start / end.
#define CSTAMP(i)                                                                  \
    do {                                                                           \
        if (threadIdx.x == 0) {                                                    \
            __builtin_amdgcn_sched_barrier(0);                                     \
            atomicAdd(&lh_stamps[32 + (i)], (unsigned long long)__builtin_amdgcn_s_memtime()); \
            __builtin_amdgcn_sched_barrier(0);                                     \
        }                                                                          \
    } while (0)
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_FLUSH(base, cnt)
#define CSTAMP(i)
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

// Workgroup barrier ordering LDS only.  __syncthreads() also releases global memory, i.e. waits
// (s_waitcnt vmcnt(0)) for every global store and prefetch load the wave has in flight; these
// kernels never hand global data between threads of a workgroup, so that wait is pure stall
// (measured: ~15k cycles per wave at the end of k_lin).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
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
__device__ __forceinline__ void d_q_from_R(const double* R, double q[4]) {
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
__device__ __forceinline__ void d_R_from_q(const double q[4], double R[9]) {
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
__device__ __forceinline__ void d_q_mul(const double* a, const double* b, double o[4]) {
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

// rotation angle of a twist (upsilon, omega): theta = |omega|
__device__ __forceinline__ double d_twist_theta(const double a[6]) {
    return sqrt(a[3] * a[3] + a[4] * a[4] + a[5] * a[5]);
}

// Sophus SE3::exp, twist (upsilon, omega) -> (q, t)   (Sophus 1.0 se3.hpp), with the
// transcendentals given: sh, ch = sin, cos(theta / 2) and st, ct = sin, cos(theta)
__device__ __forceinline__ void d_se3_exp_trig(const double a[6], double sh, double ch, double st, double ct, double q[4],
                                      double t[3]) {
    const double eps = 1e-10;
    const double* w = a + 3;
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const double th = sqrt(th2);
    double im, re;
    if (th < eps) {
        const double th4 = th2 * th2;
        im = 0.5 - (1.0 / 48.0) * th2 + (1.0 / 3840.0) * th4;
        re = 1.0 - (1.0 / 8.0) * th2 + (1.0 / 384.0) * th4;
    } else {
        im = sh / th;
        re = ch;
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
        const double c1 = (1.0 - ct) / th2;
        const double c2 = (th - st) / (th2 * th);
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

// VertexPose::add (lego_types.h, problem.cpp:433-455): estimate_ = (SE3::exp(dx) * SE3(estimate_)).matrix(),
// the candidate [R|t] (row-major, 12) from the committed one Tc and the pose step dx (translation-first
// twist; a non-finite step is skipped, as VertexPose::add's guard does).
__device__ __forceinline__ void d_pose_candidate(const double (&Tc)[12], const double* dx, double (&To)[12]) {
    double up[6];
    bool bad = false;
#pragma unroll
    for (int a = 0; a < 6; ++a) { up[a] = dx[a]; bad |= !isfinite(up[a]); }
    if (bad) {
#pragma unroll
        for (int a = 0; a < 6; ++a) up[a] = 0.0;
    }
    const double th = d_twist_theta(up);
    double sh, ch, st, ct;
    sincos(0.5 * th, &sh, &ch);
    sincos(th, &st, &ct);
    double qe[4], te[3], qT[4], qn[4], tr[3], Rn[9];
    d_se3_exp_trig(up, sh, ch, st, ct, qe, te);
    const double Rc[9] = {Tc[0], Tc[1], Tc[2], Tc[4], Tc[5], Tc[6], Tc[8], Tc[9], Tc[10]};
    d_q_from_R(Rc, qT);
    const double tc[3] = {Tc[3], Tc[7], Tc[11]};
    d_q_mul(qe, qT, qn);
    d_q_rotate(qe, tc, tr);
    d_R_from_q(qn, Rn);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        To[4 * i] = Rn[3 * i]; To[4 * i + 1] = Rn[3 * i + 1]; To[4 * i + 2] = Rn[3 * i + 2];
        To[4 * i + 3] = te[i] + tr[i];
    }
}

struct EdgeEval {
    double r0, r1, e2, rho0, rho1, rho2;
    double W00, W01, W10, W11;
    double Jp[12];   // 2 x 6, translation-first twist (lego_types.h:246-248)
    double Jl[6];    // 2 x 3
};

// the camera point ext (T X) of computeResidual (lego_types.h:213).  An extrinsic rotation that is
// exactly the identity is skipped: the quaternion rotation by (1, 0, 0, 0) returns its input exactly.
__device__ __forceinline__ void edge_pc(const double* __restrict__ pt, const double* __restrict__ e, bool ext_id,
                                        bool ext_rot, const double X[3], double Pc[3]) {
    double Pb[3];
    d_q_rotate(pt + LH_PT_QT, X, Pb);
#pragma unroll
    for (int i = 0; i < 3; ++i) Pb[i] = Pb[i] + pt[LH_PT_TT + i];
    if (ext_id) {
#pragma unroll
        for (int i = 0; i < 3; ++i) Pc[i] = Pb[i];       // identity quaternion and zero t: exact
    } else if (ext_rot) {
#pragma unroll
        for (int i = 0; i < 3; ++i) Pc[i] = Pb[i] + e[4 + i];
    } else {
        d_q_rotate(e, Pb, Pc);
#pragma unroll
        for (int i = 0; i < 3; ++i) Pc[i] = Pc[i] + e[4 + i];
    }
}

// residual_ = z - pi(K Pc), pi(q) = q / (q_z + 1e-18)   (lego_types.h:200-216), from the camera point
__device__ __forceinline__ void edge_res_pc(const double Pc[3], double u, double v, const lh_params& prm, double& r0,
                                            double& r1) {
    const double fx = prm.K[0], fy = prm.K[1], cx = prm.K[2], cy = prm.K[3];
    double p0 = fx * Pc[0] + cx * Pc[2];                  // + 0 * Pc[1]: exact
    double p1 = fy * Pc[1] + cy * Pc[2];
    const double den = Pc[2] + 1e-18;
    p0 /= den;
    p1 /= den;
    r0 = u - p0;
    r1 = v - p1;
}
// the whole residual, Pc = ext (T X) returned
__device__ __forceinline__ void edge_residual(const double* __restrict__ pt, const double* __restrict__ e, bool ext_id,
                                              bool ext_rot, const double X[3], double u, double v, const lh_params& prm,
                                              double& r0, double& r1, double Pc[3]) {
    edge_pc(pt, e, ext_id, ext_rot, X, Pc);
    edge_res_pc(Pc, u, v, prm, r0, r1);
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
        // gate_mode 1 (diagnostic): the analytically-zero residue of an outlier edge counts as 0
        if (E.rho1 + 2 * E.rho2 * E.e2 > 0.0 && !(prm.gate_mode == 1 && E.e2 > d2)) {
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

// EdgeProjection::computeJacobians (lego_types.h:218-254).  The reference evaluates them at
// ((ext T) X) and the residual at (ext (T X)); here both use the residual's point, which differs
// in rounding only (the Jacobians are not on the bitwise-mirrored path, and the back substitution
// re-derives exactly the Jacobians its linearisation used).  j_i's structural zeros J(0,1) and
// J(1,0) (lego_types.h:247-248) are left out of every product (lin_blocks); Jp[1], Jp[6] unset.
__device__ __forceinline__ void edge_jac_pc(const double Pc[3], const double* __restrict__ Rt,
                                            const double* __restrict__ e, bool ext_rot, const lh_params& prm,
                                            double Jp[12], double Jl[6]) {
    const double fx = prm.K[0], fy = prm.K[1];
    const double x = Pc[0], y = Pc[1], z = Pc[2];
    const double zi = fast_rcp(z + 1e-18);
    const double zi2 = zi * zi;
    Jp[0] = -fx * zi;              Jp[1] = 0.0;                  Jp[2] = fx * x * zi2;
    Jp[3] = fx * x * y * zi2;      Jp[4] = -fx - fx * x * x * zi2; Jp[5] = fx * y * zi;
    Jp[6] = 0.0;                   Jp[7] = -fy * zi;             Jp[8] = fy * y * zi2;
    Jp[9] = fy + fy * y * y * zi2; Jp[10] = -fy * x * y * zi2;   Jp[11] = -fy * x * zi;
    // j_j = (j_i(:, 0:3) * ext.rotationMatrix()) * T.rotationMatrix()
    double A[6];
    if (ext_rot) {   // J * I: exact
        A[0] = Jp[0]; A[1] = 0.0; A[2] = Jp[2]; A[3] = 0.0; A[4] = Jp[7]; A[5] = Jp[8];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            Jl[j] = A[0] * Rt[j] + A[2] * Rt[6 + j];
            Jl[3 + j] = A[4] * Rt[3 + j] + A[5] * Rt[6 + j];
        }
    } else {
        const double* Re = e + 7;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            A[j] = Jp[0] * Re[j] + Jp[2] * Re[6 + j];
            A[3 + j] = Jp[7] * Re[3 + j] + Jp[8] * Re[6 + j];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                Jl[3 * i + j] = A[3 * i] * Rt[j] + A[3 * i + 1] * Rt[3 + j] + A[3 * i + 2] * Rt[6 + j];
    }
}

// ---- lh_options.precision = LH_PREC_FP32_RESID (BASELINE config 3's "fp32 residuals + fp64
//      accumulate"): the Jacobians (camera point, projection derivative, chain through the extrinsic and
//      the pose rotation) in float, widened to double before any product that is summed.  The residual,
//      the Huber weight, rho0, chi2, b and the gain ratio stay the fp64 mirror of the reference's
//      arithmetic: a float residual carries ~3e-5 px of rounding, which decides LM
//      steps on weakly conditioned windows.  The step is Gauss-Newton on a Jacobian
//      rounded to float: parity to tolerance (tests/test_precision.py). ----
__device__ __forceinline__ void q_rotate_f(const double* q, const float v[3], float o[3]) {
    const float w = (float)q[0], x = (float)q[1], y = (float)q[2], z = (float)q[3];
    const float u0 = 2.0f * (y * v[2] - z * v[1]), u1 = 2.0f * (z * v[0] - x * v[2]), u2 = 2.0f * (x * v[1] - y * v[0]);
    o[0] = v[0] + w * u0 + (y * u2 - z * u1);
    o[1] = v[1] + w * u1 + (z * u0 - x * u2);
    o[2] = v[2] + w * u2 + (x * u1 - y * u0);
}

// RES: residual and robust weight into E (else E's W is the caller's); JAC: Jacobians into E
template <bool RES, bool JAC>
__device__ __forceinline__ void edge_eval_f(const double* __restrict__ pt, const double* __restrict__ e, bool ext_id,
                                            bool ext_rot, const double X[3], double u, double v, const lh_params& prm,
                                            EdgeEval& E) {
    const float Xf[3] = {(float)X[0], (float)X[1], (float)X[2]};
    float Pc[3];
    q_rotate_f(pt + LH_PT_QT, Xf, Pc);
#pragma unroll
    for (int i = 0; i < 3; ++i) Pc[i] += (float)pt[LH_PT_TT + i];
    if (!ext_id) {
        if (!ext_rot) {
            const float Pb[3] = {Pc[0], Pc[1], Pc[2]};
            q_rotate_f(e, Pb, Pc);
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) Pc[i] += (float)e[4 + i];
    }
    const float fx = (float)prm.K[0], fy = (float)prm.K[1];
    const float zi = 1.0f / (Pc[2] + 1e-18f);
    if (RES) {
        const float cx = (float)prm.K[2], cy = (float)prm.K[3];
        const float r0 = (float)u - (fx * Pc[0] + cx * Pc[2]) * zi, r1 = (float)v - (fy * Pc[1] + cy * Pc[2]) * zi;
        const float e2 = r0 * r0 + r1 * r1;
        float rho0 = e2, rho1 = 1.0f, rho2 = 0.0f, W00 = 1.0f, W01 = 0.0f, W11 = 1.0f;
        const float delta = (float)prm.huber_delta;
        if (prm.huber_delta > 0.0) {
            const float d2 = delta * delta;
            if (!(e2 <= d2)) {
                const float sq = sqrtf(e2);
                rho0 = 2.0f * sq * delta - d2;
                rho1 = delta / sq;
                rho2 = -0.5f * rho1 / e2;
            }
            W00 = rho1; W11 = rho1;
            if (rho1 + 2.0f * rho2 * e2 > 0.0f && !(prm.gate_mode == 1 && e2 > d2)) {
                const float s2 = 2.0f * rho2;
                W00 += s2 * r0 * r0;
                W01 = s2 * r0 * r1;
                W11 += s2 * r1 * r1;
            }
        }
        E.r0 = r0; E.r1 = r1; E.e2 = e2; E.rho0 = rho0; E.rho1 = rho1; E.rho2 = rho2;
        E.W00 = W00; E.W01 = W01; E.W10 = W01; E.W11 = W11;
    }
    if (JAC) {
        const float x = Pc[0], y = Pc[1], zi2 = zi * zi;
        float J[12];
        J[0] = -fx * zi;               J[1] = 0.0f;                   J[2] = fx * x * zi2;
        J[3] = fx * x * y * zi2;       J[4] = -fx - fx * x * x * zi2; J[5] = fx * y * zi;
        J[6] = 0.0f;                   J[7] = -fy * zi;               J[8] = fy * y * zi2;
        J[9] = fy + fy * y * y * zi2;  J[10] = -fy * x * y * zi2;    J[11] = -fy * x * zi;
        float A[6];
        if (ext_rot) {
            A[0] = J[0]; A[1] = 0.0f; A[2] = J[2]; A[3] = 0.0f; A[4] = J[7]; A[5] = J[8];
        } else {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                A[j] = J[0] * (float)e[7 + j] + J[2] * (float)e[13 + j];
                A[3 + j] = J[7] * (float)e[10 + j] + J[8] * (float)e[13 + j];
            }
        }
        const double* Rt = pt + LH_PT_RT;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                E.Jl[3 * i + j] = (double)(A[3 * i] * (float)Rt[j] + A[3 * i + 1] * (float)Rt[3 + j] + A[3 * i + 2] * (float)Rt[6 + j]);
#pragma unroll
        for (int k = 0; k < 12; ++k) E.Jp[k] = (double)J[k];
    }
}

// J(r, a) of j_i (2 x 6) is structurally zero: J(0, 1), J(1, 0)
__device__ __forceinline__ constexpr bool jz(int r, int a) { return (r == 0 && a == 1) || (r == 1 && a == 0); }

// Jp(:, a) . (x0, x1) without the structural zero
__device__ __forceinline__ double jdot(const double* Jp, int a, double x0, double x1) {
    if (jz(0, a)) return Jp[6 + a] * x1;
    if (jz(1, a)) return Jp[a] * x0;
    return Jp[a] * x0 + Jp[6 + a] * x1;
}

// The per-edge blocks of the linearisation (problem.cpp:285-331): H_ll, b_l, H_pl into registers,
// H_pp (21) and b_p (6) into the lane's row of the pose-sum image.  WI: every live edge of the wave
// is an inlier, so W = I and dr = 1 exactly, and W J = J.
template <bool WI>
__device__ __forceinline__ void lin_blocks(const EdgeEval& E, bool pfixed, double dr, double (&hll)[6],
                                           double (&bl)[3], double (&hpl)[18], double* __restrict__ trow) {
    const double* Jp = E.Jp;
    const double* Jl = E.Jl;
    double WJl[6];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        WJl[c] = WI ? Jl[c] : E.W00 * Jl[c] + E.W01 * Jl[3 + c];
        WJl[3 + c] = WI ? Jl[3 + c] : E.W10 * Jl[c] + E.W11 * Jl[3 + c];
    }
    hll[0] = Jl[0] * WJl[0] + Jl[3] * WJl[3];
    hll[1] = Jl[0] * WJl[1] + Jl[3] * WJl[4];
    hll[2] = Jl[0] * WJl[2] + Jl[3] * WJl[5];
    hll[3] = Jl[1] * WJl[1] + Jl[4] * WJl[4];
    hll[4] = Jl[1] * WJl[2] + Jl[4] * WJl[5];
    hll[5] = Jl[2] * WJl[2] + Jl[5] * WJl[5];
    const double dr0 = WI ? E.r0 : dr * E.r0, dr1 = WI ? E.r1 : dr * E.r1;   // rho' r
#pragma unroll
    for (int c = 0; c < 3; ++c) bl[c] = -(Jl[c] * dr0 + Jl[3 + c] * dr1);
    if (pfixed) return;
    if (WI) {
        // H_pp(a, b) = sum over the rows r where neither J(r, a) nor J(r, b) is a structural zero
        int k = 0;
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
            for (int b = a; b < 6; ++b) {
                const bool u0 = !jz(0, a) && !jz(0, b), u1 = !jz(1, a) && !jz(1, b);
                trow[k++] = u0 && u1 ? Jp[a] * Jp[b] + Jp[6 + a] * Jp[6 + b]
                                     : (u0 ? Jp[a] * Jp[b] : (u1 ? Jp[6 + a] * Jp[6 + b] : 0.0));
            }
    } else {
        double WJp[12];   // W J_p, column b: W (J(0, b), J(1, b)) with J's zero left out
#pragma unroll
        for (int b = 0; b < 6; ++b) {
            WJp[b] = jz(1, b) ? E.W00 * Jp[b] : (jz(0, b) ? E.W01 * Jp[6 + b] : E.W00 * Jp[b] + E.W01 * Jp[6 + b]);
            WJp[6 + b] = jz(1, b) ? E.W10 * Jp[b] : (jz(0, b) ? E.W11 * Jp[6 + b] : E.W10 * Jp[b] + E.W11 * Jp[6 + b]);
        }
        int k = 0;
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
            for (int b = a; b < 6; ++b) trow[k++] = jdot(Jp, a, WJp[b], WJp[6 + b]);
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) {
#pragma unroll
        for (int c = 0; c < 3; ++c) hpl[3 * a + c] = jdot(Jp, a, WJl[c], WJl[3 + c]);
        trow[21 + a] = -jdot(Jp, a, dr0, dr1);
    }
}

// LDS strides of k_lin's window pose tables and landmark-record stage, padded off the global
// ones so the entries lanes read at once fall in distinct bank groups: 26 doubles = 52 dwords puts
// 16 (slot, camera) entries on 16 distinct 4-bank groups (24 gave 4), 18 = 36 dwords puts the 8
// records of a sub-batch on 8 (16 gave 2).  Both keep 16-byte alignment for b128 loads.
#define LH_PT_LDS 26
#define LH_REC_LDS 18

template <int T>
struct LinCfg {
    static constexpr int NT = T * (T + 1) / 2;          // upper MFMA tiles of the window
    // G row stride: >= 16T and = 16 mod 32 doubles (conflict-free b64 fragment loads)
    static constexpr int GS = (T == 1) ? 16 : (T <= 3 ? 48 : (T <= 5 ? 80 : 112));
    static constexpr int UMAX = (16 * T) / 6;           // window poses that fit 16T rows
    // the chunk slab as combined in LDS: NT tiles | UMAX x 33 per-pose sums | 4 scalars (written out
    // as pair rows and the chunk scalars)
    static constexpr int LS_TASK = NT * 256, LS_SC = LS_TASK + UMAX * LH_TASKS, LS = LS_SC + 8;
    // per-wave LDS scratch: pose-sum image [slot][landmark][33], G image [24][GS], the record
    // stage (8 x LH_REC_LDS), and (over the 4 waves) the two combine slabs
    static constexpr int A_ = UMAX * LH_SB_LM * LH_TASKS, B_ = 3 * LH_SB_LM * GS, C_ = (2 * LS + 3) / 4;
    static constexpr int SCR = ((A_ > B_ ? (A_ > C_ ? A_ : C_) : (B_ > C_ ? B_ : C_)) + 1) & ~1;
};

// butterfly sum over the aligned lane group of G = 1 << lg lanes (every lane gets the total):
// v + v[lane^1], + [lane^2], + [lane^4], ... in that order.  Partners within a 16-lane row come
// through DPP (plain VALU: quad_perm for ^1 and ^2, row rotations for ^4 and ^8); ^16 and ^32
// through the permlane swaps.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(x >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// v + v[lane ^ 16] and v + v[lane ^ 32] by the gfx950 half-row / half-wave swaps (plain VALU, no LDS
// round trip as ds_bpermute takes).  With both operands v, permlane16_swap returns v[lane & ~16] and
// v[lane | 16], permlane32_swap v[lane & 31] and v[32 + (lane & 31)]: their sum is v + the partner in
// every lane (IEEE addition commutes, so the bits are those of v + partner).
__device__ __forceinline__ double xor16_sum(double v) {
    const long long x = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(x >> 32), (unsigned)(x >> 32), false, false);
    return __longlong_as_double(((long long)hi[0] << 32) | lo[0]) + __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ double xor32_sum(double v) {
    const long long x = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)x, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(x >> 32), (unsigned)(x >> 32), false, false);
    return __longlong_as_double(((long long)hi[0] << 32) | lo[0]) + __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}

// N values at once: one uniform branch per level and N independent DPP + add chains per level
// (a sum at a time serialises the branches and the DPP latencies)
template <int N>
__device__ __forceinline__ void group_sum(double (&v)[N], int lg) {
    if (lg >= 1) {                                          // quad_perm [1,0,3,2]: lane ^ 1
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] += dpp_d<0xB1>(v[i]);
    }
    if (lg >= 2) {                                          // quad_perm [2,3,0,1]: lane ^ 2
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] += dpp_d<0x4E>(v[i]);
    }
    if (lg >= 3) {                                          // lane ^ 4: row_ror 12 / row_ror 4
        const bool up = (__lane_id() & 4) != 0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const double a = dpp_d<0x12C>(v[i]), b = dpp_d<0x124>(v[i]);
            v[i] += up ? b : a;
        }
    }
    if (lg >= 4) {                                          // row_ror 8: lane ^ 8
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] += dpp_d<0x128>(v[i]);
    }
    if (lg >= 5) {
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = xor16_sum(v[i]);
    }
    if (lg >= 6) {
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = xor32_sum(v[i]);
    }
}

// the whole-wave butterfly in the other order, v + v[lane ^ 32], then ^16, ^8, ^4, ^2, ^1: the bits of the
// `v += __shfl_xor(v, off)` loop over off = 32 .. 1 (k_reduce's scalar sums) in plain VALU (ds_bpermute takes LDS
// bandwidth, which a batch's 32 sums per wave exhausted)
template <int N>
__device__ __forceinline__ void wave_sum_desc(double (&v)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = xor32_sum(v[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = xor16_sum(v[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += dpp_d<0x128>(v[i]);
    const bool up = (__lane_id() & 4) != 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const double a = dpp_d<0x12C>(v[i]), b = dpp_d<0x124>(v[i]);
        v[i] += up ? b : a;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += dpp_d<0x4E>(v[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += dpp_d<0xB1>(v[i]);
}

// max over the wave, every lane gets it: DPP within 16-lane rows, then the permlane swaps
__device__ __forceinline__ double wave_max(double v) {
    v = fmax(v, dpp_d<0xB1>(v));                                            // ^1
    v = fmax(v, dpp_d<0x4E>(v));                                            // ^2
    v = fmax(v, (__lane_id() & 4) ? dpp_d<0x124>(v) : dpp_d<0x12C>(v));     // ^4
    v = fmax(v, dpp_d<0x128>(v));                                           // ^8
    const long long x = __double_as_longlong(v);
    auto lo = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
    auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(x >> 32), (unsigned)(x >> 32), false, false);
    v = fmax(__longlong_as_double(((long long)hi[0] << 32) | lo[0]), __longlong_as_double(((long long)hi[1] << 32) | lo[1]));
    const long long y = __double_as_longlong(v);
    lo = __builtin_amdgcn_permlane32_swap((unsigned)y, (unsigned)y, false, false);
    hi = __builtin_amdgcn_permlane32_swap((unsigned)(y >> 32), (unsigned)(y >> 32), false, false);
    return fmax(__longlong_as_double(((long long)hi[0] << 32) | lo[0]), __longlong_as_double(((long long)hi[1] << 32) | lo[1]));
}

// k_lin's outputs (pair rows, per-edge rho0, landmark records) are read by later kernels only.  Stored
// plain, they sit dirty in the XCD's L2 and the kernel's end-of-launch release writes them back
// (~B / 6 TB/s at the boundary, MI355X_MICROARCH.md "boundary").  Write-through (sc1) stores leave no
// dirty line behind: k_lin 37.4 -> 36.2 us per trial launch.  LH_WT / LH_WT_REC = 0
// restore plain stores (A/B builds).
#ifndef LH_WT
#define LH_WT 1
#endif
#ifndef LH_WT_REC
#define LH_WT_REC 1
#endif

__device__ __forceinline__ void st_out(double* p, double v) {
    if constexpr (LH_WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
// k_reduce's outputs (the reduced system, its LDS images) likewise, read by the controller that follows
#ifndef LH_WT_RED
#define LH_WT_RED 1   // k_reduce 6.86 / 6.86 -> 6.71 / 6.66 us, k_ctrl +0.06 (same-box A/B, profiles/r05s_ab_wt_reduce.txt)
#endif
__device__ __forceinline__ void st_red(double* p, double v) {
    if constexpr (LH_WT_RED) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
// a landmark record's 16-byte pieces (rec_rsrc: a buffer descriptor over the record buffer)
__device__ __forceinline__ void st_rec2(double2* p, double2 v, __amdgpu_buffer_rsrc_t rsrc, const double* base) {
    if constexpr (LH_WT_REC) {
        const int off = (int)((const char*)p - (const char*)base);
        typedef int v4i __attribute__((ext_vector_type(4)));
        v4i x;
        __builtin_memcpy(&x, &v, 16);
        __builtin_amdgcn_raw_buffer_store_b128(x, rsrc, off, 0, 16);   // aux 16: sc1 (write-through)
    } else {
        *p = v;
    }
}

static_assert(offsetof(lh_chunk, sb_end) == 4 && offsetof(lh_chunk, U) == 8, "k_lin reads the chunk header as dwords");

// ---- back-substitution of the pending pose step (problem.cpp:426-429) for one sub-batch: the lane's edge term
//      J_l^T W J_p dx (at the committed linearisation: pt the committed pose table, d the slot's step), summed over
//      the landmark's lane group, then the landmark's update from its cached factor cl (VertexXYZ::add) and the
//      lead lane's gain-scale term (isGoodStepInLM's scale) ----
// (1) the edge's weight and Jacobians at the committed linearisation: pt the committed pose table, X the
//     committed landmark (a live edge only)
template <bool F32>
__device__ __forceinline__ void backsub_jac(const double* __restrict__ pt, const double* __restrict__ e, bool ext_id,
                                            bool ext_rot, double u, double v, int wfl, const double (&X)[3],
                                            const lh_params& prm, EdgeEval& E) {
    if constexpr (F32) {   // fp64 residual and weight (as below), fp32 Jacobians
        if (wfl) {
            E.W00 = 1.0; E.W01 = 0.0; E.W10 = 0.0; E.W11 = 1.0;
        } else {
            double Pc[3];
            edge_residual(pt, e, ext_id, ext_rot, X, u, v, prm, E.r0, E.r1, Pc);
            edge_robust(E, prm);
        }
        edge_eval_f<false, true>(pt, e, ext_id, ext_rot, X, u, v, prm, E);
    } else {
        double Pc[3];
        if (wfl) {   // an inlier at the committed linearisation: W = I, no residual needed
            E.W00 = 1.0; E.W01 = 0.0; E.W10 = 0.0; E.W11 = 1.0;
            edge_pc(pt, e, ext_id, ext_rot, X, Pc);
        } else {
            edge_residual(pt, e, ext_id, ext_rot, X, u, v, prm, E.r0, E.r1, Pc);
            edge_robust(E, prm);
        }
        edge_jac_pc(Pc, pt + LH_PT_RT, e, ext_rot, prm, E.Jp, E.Jl);
    }
}
// (2) the step d's term J_l^T W J_p d over the landmark's lane group, the landmark's update from its cached factor
//     cl, and the lead lane's gain-scale term at lambda.  The multiply-adds are explicit fused ones: where the
//     compiler contracts a * b + c * d it picks the product to fuse by the products' use counts, which depend on the
//     code around the call, and the batch path (one Jacobian, several steps) and the trial path must round alike.
//     The forms below are the ones the trial path was compiled to (the pre-split build's bits, scripts/lib_bitwise.py).
__device__ __forceinline__ void backsub_apply(const EdgeEval& E, bool live, const double* __restrict__ d, int lg,
                                              bool lmok, bool lead, const double (&cl)[12], double lambda,
                                              const lh_params& prm, double (&X)[3], double& scale_acc) {
    double v3[3] = {0.0, 0.0, 0.0};
    if (live) {
        double jd0 = 0.0, jd1 = 0.0;
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            if (!jz(0, a)) jd0 = __builtin_fma(E.Jp[a], d[a], jd0);
            if (!jz(1, a)) jd1 = __builtin_fma(E.Jp[6 + a], d[a], jd1);
        }
        const double y0 = __builtin_fma(E.W01, jd1, E.W00 * jd0), y1 = __builtin_fma(E.W11, jd1, E.W10 * jd0);
#pragma unroll
        for (int c = 0; c < 3; ++c) v3[c] = __builtin_fma(E.Jl[c], y0, E.Jl[3 + c] * y1);
    }
    group_sum(v3, lg);
    const double s0 = v3[0], s1 = v3[1], s2 = v3[2];
    if (lmok) {
        // the cached factor holds 1/L_ii on the diagonal
        const double i00 = cl[0], l10 = cl[1], i11 = cl[2], l20 = cl[3], l21 = cl[4], i22 = cl[5];
        const double b0 = cl[6], b1 = cl[7], b2 = cl[8];
        const double t0 = b0 - s0, t1 = b1 - s1, t2 = b2 - s2;
        const double y0 = t0 * i00, y1 = __builtin_fma(-l10, y0, t1) * i11;
        const double y2 = __builtin_fma(-l21, y1, __builtin_fma(-l20, y0, t2)) * i22;
        double d2 = y2 * i22, d1 = __builtin_fma(-l21, d2, y1) * i11;
        double d0 = __builtin_fma(-l20, d2, __builtin_fma(-l10, d1, y0)) * i00;
        if (prm.guard && !(i00 == i00)) { d0 = d1 = d2 = 0.0; }   // skipped degenerate landmark
        double x0 = X[0], x1 = X[1], x2 = X[2];
        if (isfinite(d0) && isfinite(d1) && isfinite(d2)) { x0 += d0; x1 += d1; x2 += d2; }   // VertexXYZ::add
        if (lead) {
            double q0, q1, q2;
            if (prm.strategy == 0) {
                q0 = __builtin_fma(lambda, d0, b0); q1 = __builtin_fma(lambda, d1, b1); q2 = __builtin_fma(lambda, d2, b2);
            } else {
                q0 = __builtin_fma(lambda * cl[9], d0, b0); q1 = __builtin_fma(lambda * cl[10], d1, b1);
                q2 = __builtin_fma(lambda * cl[11], d2, b2);
            }
            const double sc = __builtin_fma(d2, q2, __builtin_fma(d0, q0, d1 * q1));
            scale_acc += sc;
        }
        X[0] = x0; X[1] = x1; X[2] = x2;
    }
}
template <bool F32>
__device__ __forceinline__ void lin_backsub(const double* __restrict__ pt, const double* __restrict__ e,
                                            const double* __restrict__ d, bool live, bool ext_id, bool ext_rot, double u,
                                            double v, int wfl, int lg, bool lmok, bool lead, const double (&cl)[12],
                                            double lambda, const lh_params& prm, double (&X)[3], double& scale_acc) {
    EdgeEval E;
    if (live) backsub_jac<F32>(pt, e, ext_id, ext_rot, u, v, wfl, X, prm, E);
    backsub_apply(E, live, d, lg, lmok, lead, cl, lambda, prm, X, scale_acc);
}

// A batch group's candidate pose tables (k_lin's batch path, all threads): item i < gn U is rung i / U's candidate
// pose of slot i % U, from the committed pose pm (slot's pose cpose[slot]) and the rung's step (LDS wd + 6 U r),
// staged in LDS cand; then item j < gn U ncam builds the table of (rung, slot, camera) into LDS tabs + per_tab r,
// as k_lin's own candidate build does.  LDS operands as offsets into the dynamic LDS; out of line, so that its
// registers are not the trial path's.
__device__ __attribute__((noinline)) void lin_cand_batch(const double* __restrict__ pm, const uint16_t* __restrict__ cpose,
                                                         int pmax1, int U, int ncam, int gn, int o_wd, int o_cand,
                                                         int o_tabs, int per_tab, int o_wext) {
    extern __shared__ __attribute__((aligned(16))) double dsm[];
    const int tid = threadIdx.x;
    for (int i = tid; i < gn * U; i += 256) {
        const int r = i / U, sl = i - r * U;
        const uint32_t pp = min((uint32_t)cpose[sl], (uint32_t)pmax1);
        double pmc[12], To[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) pmc[k] = pm[pp * 12 + k];
        d_pose_candidate(pmc, dsm + o_wd + 6 * U * r + 6 * sl, To);
#pragma unroll
        for (int k = 0; k < 12; ++k) dsm[o_cand + 12 * i + k] = To[k];
    }
    lds_barrier();
    for (int i = tid; i < gn * U * ncam; i += 256) {
        const int r = i / (U * ncam), j = i - r * U * ncam, sl = j / ncam, c = j - sl * ncam;
        double To[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) To[k] = dsm[o_cand + 12 * (r * U + sl) + k];
        d_pose_table(To, dsm + o_wext + c * LH_EXT, dsm + o_tabs + per_tab * r + (sl * ncam + c) * LH_PT_LDS);
    }
}

#ifndef LH_LIN_OCC
#define LH_LIN_OCC 2   // k_lin<T <= 3> workgroups per CU the registers are budgeted for
#endif
template <int T, bool TRIAL, bool F32>
__global__ __launch_bounds__(256, (T <= 3) ? LH_LIN_OCC : 1) void k_lin(
    const lh_chunk* __restrict__ chunks, const lh_subbatch* __restrict__ sbs, const float* __restrict__ obs_uv,
    const uint32_t* __restrict__ obs_meta, double* __restrict__ rec, double* __restrict__ pose_tab,
    const double* __restrict__ ext, const lh_ctrl* __restrict__ ctrl, const double* __restrict__ dxp,
    double* __restrict__ edge_rho, double* __restrict__ rows, double* __restrict__ csc,
    const uint32_t* __restrict__ crow, uint8_t* __restrict__ wflag, long nslots,
    lh_params prm, int nrec, const uint64_t* __restrict__ fixed_bits, int chunk_base,
    double* __restrict__ pose_mat, int writer, lh_reset_args rst) {
    using Cfg = LinCfg<T>;
    extern __shared__ __attribute__((aligned(16))) double dsm[];

    // The prologue's global loads go out in two dependent rounds: (1) the controller words and the
    // chunk header (scalar), then every independent vector load, the first sub-batch's prefetch
    // included; (2) the pose-table and pose-step values, whose addresses need the chunk's pose slots.
    // Written as per-element loops, each loop iteration waited for its own loads (ten serialised
    // round trips before the first sub-batch).
    // the initial linearisation restarts the solve (rst, its writer block below): the controller is not read
    const int done = TRIAL ? __builtin_amdgcn_readfirstlane(ctrl->done) : 0;
    const int cur = TRIAL ? __builtin_amdgcn_readfirstlane(ctrl->cur) : 0;
    // the re-linearisation of an evaluate-only acceptance (ctrl->relin, ctrl_lm_step): no back substitution and
    // no candidate; the committed landmarks and pose tables are linearised into the candidate side, which the
    // chain's decision commits (the writer copies the committed poses and tables across first)
    const bool relin = TRIAL && __builtin_amdgcn_readfirstlane(ctrl->relin) != 0;
    // the evo word: a trial of the final LM iteration or after a rejection (ctrl_lm_step) only evaluates, and above
    // its low byte the rung count of a batch of such trials (k_reduce's decision; the batch path after the tables)
    const int evw = TRIAL ? __builtin_amdgcn_readfirstlane(ctrl->evo) : 0;
    const int nbatch = max(evw >> 8, 1);
    // the pending step: lambda-ladder rung ctrl->lad's (the rung the last decision moved to; 0 after a factor)
    if (TRIAL) dxp += (size_t)__builtin_amdgcn_readfirstlane(ctrl->lad) * prm.n;
    // The candidate poses of a trial (VertexPose::add of the step k_ctrl solved) are built here, not in
    // the serial controller: every chunk builds its own window's candidate pose tables (wave 3, below),
    // and block 0 of one launch per trial (writer) stores every candidate pose and its tables, which a
    // later trial reads as committed and the caller as the result.
    if (!TRIAL && writer && blockIdx.x == 0) {   // the restart (what a separate reset kernel did)
        // (ctrl and dxp are read-only to every trial launch; in this launch no other block reads them, and
        // the controller words written here are read by the later kernels of the chain)
        int* c = reinterpret_cast<int*>(const_cast<lh_ctrl*>(ctrl));
        for (int i = threadIdx.x; i < (int)(sizeof(lh_ctrl) / sizeof(int)); i += 256) c[i] = 0;   // cur = 0
        for (int i = threadIdx.x; i < rst.nqt; i += 256) pose_mat[i] = rst.qt_init[i];
        for (int i = threadIdx.x; i < rst.nptab; i += 256) pose_tab[i] = rst.ptab_init[i];
        for (int i = threadIdx.x; i < rst.ndxp; i += 256) const_cast<double*>(dxp)[i] = 0.0;
        return;
    }
    if (TRIAL && writer && blockIdx.x == 0) {
        if (done || nbatch > 1) return;   // (a batch writes no candidate: its accepted rung is re-run in full)
        const int P = prm.P, nc = prm.ncam, cnd = 1 - cur;
        if (relin) {
            for (int i = threadIdx.x; i < P * 12; i += 256) pose_mat[(size_t)cnd * P * 12 + i] = pose_mat[(size_t)cur * P * 12 + i];
            for (int i = threadIdx.x; i < P * nc * LH_PT; i += 256)
                pose_tab[(size_t)cnd * P * nc * LH_PT + i] = pose_tab[(size_t)cur * P * nc * LH_PT + i];
            return;
        }
        for (int p = threadIdx.x; p < P; p += 256) {
            double Tc[12], To[12];
#pragma unroll
            for (int i = 0; i < 12; ++i) Tc[i] = pose_mat[(size_t)cur * P * 12 + p * 12 + i];
            d_pose_candidate(Tc, dxp + 6 * p, To);
#pragma unroll
            for (int i = 0; i < 12; ++i) pose_mat[(size_t)cnd * P * 12 + p * 12 + i] = To[i];
            for (int c = 0; c < nc; ++c)
                d_pose_table(To, ext + LH_EXT * c, pose_tab + (size_t)cnd * P * nc * LH_PT + (p * nc + c) * LH_PT);
        }
        return;
    }
    const int chunk = chunk_base + blockIdx.x - (writer ? 1 : 0);
    // a trial of the final LM iteration (ctrl->evo, ctrl_lm_step): back substitution and the
    // candidate's evaluation only (landmark positions, rho0 per edge, chi2 and the gain scale)
    const bool evo = evw != 0;
    const double lambda = TRIAL ? ctrl->lambda : 0.0;
    const uint32_t* __restrict__ chw = reinterpret_cast<const uint32_t*>(chunks + chunk);
    const uint32_t sb_begin = __builtin_amdgcn_readfirstlane(chw[0]), sb_end = __builtin_amdgcn_readfirstlane(chw[1]);
    const int U = (int)(__builtin_amdgcn_readfirstlane(chw[2]) & 0xffu);   // lh_chunk: {sb_begin, sb_end, U, T, ...}
    const uint32_t item_base = chunks[chunk].item_base;
    if (done) return;
    const int cand = 1 - cur;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar loads, scalar loop
    const int ncam = prm.ncam;
    const int PT = prm.P * ncam * LH_PT;
    const uint16_t* __restrict__ cpose = chunks[chunk].pose;

    double* scr = dsm + wave * Cfg::SCR;
    // the chunk's window, LDS-resident: committed and candidate pose tables per (slot, camera),
    // the pending pose step per slot, the camera extrinsics
    double* wt_c = dsm + LH_WAVES * Cfg::SCR;
    double* wt_n = wt_c + Cfg::UMAX * ncam * LH_PT_LDS;     // a chunk of T tiles has U <= UMAX poses
    double* wdx = wt_n + Cfg::UMAX * ncam * LH_PT_LDS;
    double* wext = wdx + Cfg::UMAX * 6;
    // after the pair-row map: the flag raised when wave 3 has built the candidate tables
    int* cflag = reinterpret_cast<int*>(wext + ncam * LH_EXT + (Cfg::UMAX * (Cfg::UMAX + 1) / 2 + 1) / 2);
    double pmc[12];
    // the wave that builds the candidate pose tables: 3 or 2 by block parity, so the two chunks sharing a
    // CU build them on different SIMDs (measured 37.7 -> 37.5 us per k_lin against wave 3 in both)
    const int cwave = LH_WAVES - 1 - (blockIdx.x & 1);

    const double2* __restrict__ rc2 = reinterpret_cast<const double2*>(rec + (size_t)cur * nrec * LH_REC);
    // piece lane & 7 of sub-batch sbx's record (lane >> 3); the initial linearisation reads only X, from the window
    auto rec_piece = [&](int sbx) -> double2 {
        if constexpr (TRIAL) {
            return rc2[(size_t)sbx * 64 + lane];
        } else {
            const int q = lane & 7, l = rst.lm_perm[sbx * LH_SB_LM + (lane >> 3)];
            if (q > 1 || l < 0) return double2{0.0, 0.0};
            const double* X = rst.lm_in + 3 * (size_t)l;
            return q == 0 ? double2{X[0], X[1]} : double2{X[2], 0.0};
        }
    };
    double* __restrict__ rn = rec + (size_t)cand * nrec * LH_REC;
    // a descriptor over both record buffers (write-through record stores, LH_WT_REC)
    const __amdgpu_buffer_rsrc_t rec_rsrc =
        __builtin_amdgcn_make_buffer_rsrc(rec, 0, (int)((size_t)2 * nrec * LH_REC * sizeof(double)), 0x00020000);

    v4d acc[Cfg::NT];
#pragma unroll
    for (int t = 0; t < Cfg::NT; ++t) acc[t] = v4d{0.0, 0.0, 0.0, 0.0};
    // per-pose sums: lane l owns the (slot, task) cells c = l + 64 i, c = 33 slot + task (all 64 lanes)
    constexpr int NCELL = (Cfg::UMAX * LH_TASKS + 63) / 64;
    double task[NCELL];
#pragma unroll
    for (int u = 0; u < NCELL; ++u) task[u] = 0.0;
    double chi_acc = 0.0, scale_acc = 0.0, maxd = 0.0, ndeg = 0.0;
    STAMP_DECL

    // prefetch of the first sub-batch: observation words and the 8 landmark records.  The
    // prefetch is unconditional (index clamped to the chunk) so the compiler can keep it in
    // flight with counted vmcnt waits across the iteration.
    const int sb_last = (int)sb_end - 1;
    int sb = (int)sb_begin + wave;
    // wflag[buffer][slot]: 1 where the linearisation that produced that buffer's state found the edge
    // an inlier (e2 <= delta^2, or no robust kernel), i.e. its robust weight W is exactly I
    const uint8_t* __restrict__ wf_c = wflag + (size_t)cur * nslots;
    uint8_t* __restrict__ wf_n = wflag + (size_t)cand * nslots;
    uint32_t meta_n;
    double u_n, v_n;
    double2 r_n;
    int wfl_n = 0;
    lh_subbatch S_n;
    {
        const int sbc = min(sb, sb_last);
        const int o = sbc * 64 + lane;
        S_n = sbs[sbc];
        meta_n = obs_meta[o];
        if (TRIAL) wfl_n = wf_c[o];
        const float2 z = reinterpret_cast<const float2*>(obs_uv)[o];   // the float pixel, widened exactly
        u_n = (double)z.x;
        v_n = (double)z.y;
        r_n = rec_piece(sbc);
    }
    {
        // round 1: the pose slot of each table element this thread copies, the extrinsics, the
        // chunk's pair rows (written by the epilogue); round 2: the table values and the pose step.
        // Every load is unconditional, its index clamped into range (a conditional load becomes a
        // branch, and the wait at its join serialises the rounds again); only the LDS writes are guarded.
        static_assert(6 * Cfg::UMAX <= 256 && Cfg::UMAX * (Cfg::UMAX + 1) / 2 <= 256 && 4 * LH_EXT <= 256,
                      "one element per thread");
        constexpr int NTAB = (Cfg::UMAX * 4 * LH_PT + 255) / 256;   // ncam <= 4
        const int per = ncam * LH_PT, ne = U * per, nrow = U * (U + 1) / 2;
        const int umax1 = max(U - 1, 0);
        const uint32_t pmax1 = (uint32_t)(prm.P - 1);
        int tsl[NTAB];
        uint32_t tp[NTAB];
#pragma unroll
        for (int k = 0; k < NTAB; ++k) {
            const int i = tid + 256 * k;
            tsl[k] = min(i / per, umax1);
            tp[k] = min((uint32_t)cpose[tsl[k]], pmax1);
        }
        const bool has_dx = TRIAL && tid < 6 * U;
        const int di = min(tid / 6, umax1);
        const uint32_t dp = min((uint32_t)cpose[di], pmax1);
        const double ev = ext[min(tid, ncam * LH_EXT - 1)];
        const uint32_t rw = crow[item_base + min(tid, max(nrow - 1, 0))];
        double tc[NTAB], tn[NTAB];
#pragma unroll
        for (int k = 0; k < NTAB; ++k) {
            const int i = tid + 256 * k;
            const size_t g = (size_t)tp[k] * per + min(max(i - tsl[k] * per, 0), per - 1);
            tc[k] = pose_tab[(size_t)cur * PT + g];
            tn[k] = TRIAL ? 0.0 : rst.ptab_init[(size_t)cand * PT + g];   // a trial builds its candidate tables
        }
        if (TRIAL && wave == cwave) {   // the committed pose of slot lane (lane < U)
            const uint32_t pp = min((uint32_t)cpose[min(lane, umax1)], pmax1);
#pragma unroll
            for (int i = 0; i < 12; ++i) pmc[i] = pose_mat[(size_t)cur * prm.P * 12 + pp * 12 + i];
        }
        const double dv = TRIAL ? dxp[6 * dp + (tid - 6 * (tid / 6))] : 0.0;
#pragma unroll
        for (int k = 0; k < NTAB; ++k) {
            const int i = tid + 256 * k;
            if (i < ne) {
                const int r = i - tsl[k] * per, ent = r / LH_PT;
                const int l = (tsl[k] * ncam + ent) * LH_PT_LDS + (r - ent * LH_PT);
                wt_c[l] = tc[k];
                if (!TRIAL) wt_n[l] = tn[k];
            }
        }
        if (has_dx) wdx[tid] = dv;
        if (tid < ncam * LH_EXT) wext[tid] = ev;
        uint32_t* wrow = reinterpret_cast<uint32_t*>(wext + ncam * LH_EXT);
        if (tid < nrow) wrow[tid] = rw;
        if (tid == 0) *cflag = 0;
    }
    lds_barrier();   // window tables
    if (TRIAL && nbatch > 1) {
        // ---- a batch: the evaluate-only trials of rungs lad .. lad + nbatch - 1 after a rejection,
        //      each evaluated as the evaluate-only path below evaluates one trial: the back substitution of the
        //      rung's step at the rung's lambda, the rung's candidate pose tables, rho0 per edge (edge_rho + r nslots)
        //      and the chunk's chi2 and gain scale (csc + (r n_chunks + chunk) 4).  The rungs of a group share one
        //      pass over the chunk's sub-batches: an edge's weight and Jacobians at the committed state are computed
        //      once, then each rung's step is applied and its candidate evaluated.  Each lane's chi2 and scale sums
        //      per rung stay in LDS (the same per-lane order as the single-trial path).  Nothing else is written:
        //      k_reduce decides the rungs in order, and the next chain re-runs an accepted rung as a full trial.
        //      LDS: the trial path's wave scratch [0, 4 SCR), free here: record stages, rung lambdas, the combine's
        //      wave totals, then per rung of a group: the lanes' sums, candidate tables, step, candidate poses. ----
        double* stg = dsm + wave * (8 * LH_REC_LDS);               // this wave's landmark-record stage
        double* lam_l = dsm + LH_WAVES * 8 * LH_REC_LDS;           // [LH_LAD] the rungs' lambdas
        double* wtot = lam_l + LH_LAD;                             // [LH_LAD][LH_WAVES][2] wave totals
        double* gbase = wtot + LH_LAD * LH_WAVES * 2;
        const int per_tab = U * ncam * LH_PT_LDS;
        const int per_rung = 2 * LH_WAVES * 64 + per_tab + 6 * U + 12 * U;
        const int avail = LH_WAVES * Cfg::SCR - (int)(gbase - dsm);
        static_assert(LH_WAVES * Cfg::SCR - (LH_WAVES * 8 * LH_REC_LDS + LH_LAD + LH_LAD * LH_WAVES * 2) >=
                          2 * LH_WAVES * 64 + Cfg::UMAX * 4 * LH_PT_LDS + 18 * Cfg::UMAX,
                      "a batch group of one rung (4 cameras) fits the wave scratch");
        const int G = max(1, min(nbatch, avail / per_rung));      // rungs per group
        double* acc_c = gbase;                                     // [G][LH_WAVES][64] chi2 per lane
        double* acc_s = acc_c + G * LH_WAVES * 64;                 // [G][LH_WAVES][64] gain scale per lane
        double* tabs = acc_s + G * LH_WAVES * 64;                  // [G][per_tab] candidate tables
        double* wd = tabs + G * per_tab;                           // [G][6 U] steps
        double* cand = wd + G * 6 * U;                             // [G][U][12] candidate poses
        if (tid == 0) {   // rung r's lambda: r more rejections' updates (ctrl_lm_step, ladder_read's order)
            double lam = lambda, ni = ctrl->ni;
            for (int r = 0; r < nbatch; ++r) {
                if (r > 0) {
                    if (prm.strategy == 0) { lam *= ni; ni *= 2.0; }
                    else lam = fmin(lam * 11.0, 1e7);
                }
                lam_l[r] = lam;
            }
        }
        for (int g0 = 0; g0 < nbatch; g0 += G) {
            const int gn = min(G, nbatch - g0);
            lds_barrier();   // (the previous group's combine is done with the LDS)
            for (int i = tid; i < gn * 6 * U; i += 256) {
                const int r = i / (6 * U), k = i - r * 6 * U;
                wd[i] = dxp[(size_t)(g0 + r) * prm.n + 6 * (size_t)min((uint32_t)cpose[k / 6], (uint32_t)(prm.P - 1)) + k % 6];
            }
            for (int i = tid; i < gn * LH_WAVES * 64; i += 256) { acc_c[i] = 0.0; acc_s[i] = 0.0; }
            lds_barrier();
            lin_cand_batch(pose_mat + (size_t)cur * prm.P * 12, cpose, prm.P - 1, U, ncam, gn, (int)(wd - dsm),
                           (int)(cand - dsm), (int)(tabs - dsm), per_tab, (int)(wext - dsm));
            lds_barrier();
            for (int sbi = (int)sb_begin + wave; sbi < (int)sb_end; sbi += LH_WAVES) {
                const lh_subbatch S = S_n;
                const int lg = S.lg, nlm = S.n_lm;
                const int ls = lane >> lg, gj = lane & ((1 << lg) - 1);
                const bool lmok = ls < nlm;
                const bool lead = gj == 0 && lmok;
                const uint32_t meta = meta_n;
                const double u = u_n, v = v_n;
                const double2 rr = r_n;
                const int wfl = wfl_n;
                const int o = sbi * 64 + lane;
                {   // the next sub-batch's words: after the wave's last one, its first again (the next group's)
                    const int sbw = sbi + LH_WAVES < (int)sb_end ? sbi + LH_WAVES : (int)sb_begin + wave;
                    const int sbn = min(sbw, sb_last);
                    const int on = sbn * 64 + lane;
                    S_n = sbs[sbn];
                    meta_n = obs_meta[on];
                    wfl_n = wf_c[on];
                    const float2 z = reinterpret_cast<const float2*>(obs_uv)[on];
                    u_n = (double)z.x;
                    v_n = (double)z.y;
                    r_n = rec_piece(sbn);
                }
                reinterpret_cast<double2*>(stg)[(lane >> 3) * (LH_REC_LDS / 2) + (lane & 7)] = rr;
                wave_sync();
                const double* myrec = stg + (ls & 7) * LH_REC_LDS;
                const double X[3] = {myrec[LH_REC_X], myrec[LH_REC_X + 1], myrec[LH_REC_X + 2]};
                double cl[12];
#pragma unroll
                for (int i = 0; i < 12; ++i) cl[i] = myrec[LH_REC_L + i];
                wave_sync();
                const bool has = (meta & LH_META_VALID) != 0u;
                const int p = LH_META_POSE(meta), cam = LH_META_CAM(meta), slot = LH_META_SLOT(meta);
                const bool pfixed = (fixed_bits[p >> 6] >> (p & 63)) & 1ull;
                const bool live = has && !pfixed;
                const double* e = wext + cam * LH_EXT;
                const bool ext_id = (prm.ext_identity >> cam) & 1;
                const bool ext_rot = (prm.ext_rot_identity >> cam) & 1;
                EdgeEval E;
                if (live) backsub_jac<F32>(wt_c + (slot * ncam + cam) * LH_PT_LDS, e, ext_id, ext_rot, u, v, wfl, X, prm, E);
                for (int r = 0; r < gn; ++r) {
                    double Xr[3] = {X[0], X[1], X[2]};
                    const int ai = (r * LH_WAVES + wave) * 64 + lane;
                    double sa = acc_s[ai];
                    backsub_apply(E, live, wd + r * 6 * U + 6 * slot, lg, lmok, lead, cl, lam_l[g0 + r], prm, Xr, sa);
                    acc_s[ai] = sa;
                    if (has) {
                        const double* pt = tabs + r * per_tab + (slot * ncam + cam) * LH_PT_LDS;
                        EdgeEval Ec;
                        double Pc[3];
                        edge_residual(pt, e, ext_id, ext_rot, Xr, u, v, prm, Ec.r0, Ec.r1, Pc);
                        edge_robust(Ec, prm);
                        st_out(edge_rho + (size_t)(g0 + r) * nslots + o, Ec.rho0);
                        acc_c[ai] = acc_c[ai] + Ec.rho0;
                    }
                }
            }
            // each rung's wave totals (the single-trial path's butterflies), then its chunk scalars in that path's
            // combine order, (w0 + w2) + (w1 + w3)
            for (int r = 0; r < gn; ++r) {
                const int ai = (r * LH_WAVES + wave) * 64 + lane;
                double t3[3] = {acc_c[ai], acc_s[ai], 0.0};
                group_sum(t3, 6);
                if (lane == 0) { wtot[(r * LH_WAVES + wave) * 2] = t3[0]; wtot[(r * LH_WAVES + wave) * 2 + 1] = t3[1]; }
            }
            lds_barrier();
            for (int i = tid; i < gn * 4; i += 256) {
                const int r = i >> 2, k = i & 3;
                const double* wt = wtot + r * LH_WAVES * 2;
                csc[((size_t)(g0 + r) * prm.n_chunks + chunk) * 4 + k] =
                    k < 2 ? (wt[0 * 2 + k] + wt[2 * 2 + k]) + (wt[1 * 2 + k] + wt[3 * 2 + k]) : 0.0;
            }
        }
        return;
    }
    // A trial's candidate pose tables (wt_n): wave cwave composes the window's candidate poses (lane = slot)
    // and their tables (lane = (slot, camera)) while the other waves start their first back
    // substitution, which needs only the committed tables; they wait on cflag before their first
    // evaluation at the candidate.  Waves 2 and 3 run one sub-batch fewer than wave 0 in most chunks.
    if (TRIAL && !relin && wave == cwave) {
        if (lane < U) {
            double To[12];
            d_pose_candidate(pmc, wdx + 6 * lane, To);
#pragma unroll
            for (int i = 0; i < 12; ++i) scr[lane * 12 + i] = To[i];
        }
        wave_sync();
        if (lane < U * ncam) {
            const int sl = lane / ncam, c = lane - sl * ncam;
            double To[12];
#pragma unroll
            for (int i = 0; i < 12; ++i) To[i] = scr[sl * 12 + i];
            d_pose_table(To, wext + c * LH_EXT, wt_n + (sl * ncam + c) * LH_PT_LDS);
        }
        __hip_atomic_store(cflag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    bool tabs_ready = !TRIAL || relin;
    const double* wt_l = relin ? wt_c : wt_n;   // the tables the edges are evaluated and linearised at

    for (; sb < (int)sb_end; sb += LH_WAVES) {
        const lh_subbatch S = S_n;       // scalar words, prefetched one sub-batch ahead (sb is wave-uniform)
        const int lg = S.lg, nlm = S.n_lm;
        const int ls = lane >> lg, gj = lane & ((1 << lg) - 1);
        const bool lmok = ls < nlm;
        const bool lead = gj == 0 && lmok;           // one lane per landmark writes its record
        const uint32_t meta = meta_n;
        const double u = u_n, v = v_n;
        const double2 rr = r_n;
        const int wfl = wfl_n;
        const int o = sb * 64 + lane;
        {
            const int sbn = min(sb + LH_WAVES, sb_last);
            const int on = sbn * 64 + lane;
            S_n = sbs[sbn];
            meta_n = obs_meta[on];
            if (TRIAL) wfl_n = wf_c[on];
            const float2 z = reinterpret_cast<const float2*>(obs_uv)[on];
            u_n = (double)z.x;
            v_n = (double)z.y;
            r_n = rec_piece(sbn);
        }
        // landmark records through LDS: lane -> its landmark's record (records LH_REC_LDS apart)
        reinterpret_cast<double2*>(scr)[(lane >> 3) * (LH_REC_LDS / 2) + (lane & 7)] = rr;
        wave_sync();
        const double* myrec = scr + (ls & 7) * LH_REC_LDS;
        double X[3] = {myrec[LH_REC_X], myrec[LH_REC_X + 1], myrec[LH_REC_X + 2]};
        double cl[12];
        if (TRIAL) {
#pragma unroll
            for (int i = 0; i < 12; ++i) cl[i] = myrec[LH_REC_L + i];
        }
        wave_sync();
        if (!evo) {
            // the pose-sum image [landmark][slot][33] starts at zero: cells without a live
            // observation then add exact zeros, and the per-slot sums need no masks or branches
            double2* z = reinterpret_cast<double2*>(scr);
            constexpr int nz = (LH_SB_LM * Cfg::UMAX * LH_TASKS) / 2;
#pragma unroll
            for (int k = 0; k < (nz + 63) / 64; ++k)
                if (k * 64 + lane < nz) z[k * 64 + lane] = double2{0.0, 0.0};
        }
        wave_sync();

        const bool has = (meta & LH_META_VALID) != 0u;
        const int p = LH_META_POSE(meta), cam = LH_META_CAM(meta), slot = LH_META_SLOT(meta);
        const bool pfixed = (fixed_bits[p >> 6] >> (p & 63)) & 1ull;
        const bool live = has && !pfixed;
        const double* e = wext + cam * LH_EXT;
        const bool ext_id = (prm.ext_identity >> cam) & 1;
        const bool ext_rot = (prm.ext_rot_identity >> cam) & 1;

        // ---- back-substitution of the pending pose step (problem.cpp:426-429) ----
        if (TRIAL && !relin)
            lin_backsub<F32>(wt_c + (slot * ncam + cam) * LH_PT_LDS, e, wdx + 6 * slot, live, ext_id, ext_rot, u, v, wfl,
                             lg, lmok, lead, cl, lambda, prm, X, scale_acc);
        STAMP(0);
        if (!tabs_ready) {   // wave-uniform: once per wave
            while (__hip_atomic_load(cflag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(1);
            tabs_ready = true;
        }

        if (evo) {   // the same evaluation as below, without the linearisation
            if (has) {
                const double* pt = wt_l + (slot * ncam + cam) * LH_PT_LDS;
                EdgeEval E;
                double Pc[3];
                edge_residual(pt, e, ext_id, ext_rot, X, u, v, prm, E.r0, E.r1, Pc);
                edge_robust(E, prm);
                st_out(edge_rho + o, E.rho0);
                chi_acc += E.rho0;
            }
            if (lead) {
                double* rw = rn + ((size_t)sb * LH_SB_LM + ls) * LH_REC;
                st_rec2(reinterpret_cast<double2*>(rw), double2{X[0], X[1]}, rec_rsrc, rec);
                st_out(rw + 2, X[2]);
            }
            continue;
        }

        // ---- evaluate and linearise at the candidate (problem.cpp:285-331, :523-526) ----
        // H_pp and b_p go straight to this lane's row of the pose-sum transpose
        double hll[6] = {0, 0, 0, 0, 0, 0}, bl[3] = {0, 0, 0};
        double hpl[18];
#pragma unroll
        for (int i = 0; i < 18; ++i) hpl[i] = 0.0;
        // [landmark][slot][33]: unique writer; a wave's 16-lane store group covers distinct cells
        double* trow = scr + ((ls & 7) * Cfg::UMAX + slot) * LH_TASKS;
        if (has) {
            const double* pt = wt_l + (slot * ncam + cam) * LH_PT_LDS;
            EdgeEval E;
            double Pc[3];
            edge_residual(pt, e, ext_id, ext_rot, X, u, v, prm, E.r0, E.r1, Pc);
            edge_robust(E, prm);
            if constexpr (F32) edge_eval_f<false, true>(pt, e, ext_id, ext_rot, X, u, v, prm, E);
            else edge_jac_pc(Pc, pt + LH_PT_RT, e, ext_rot, prm, E.Jp, E.Jl);
            st_out(edge_rho + o, E.rho0);
            chi_acc += E.rho0;
            const bool inl = prm.huber_delta <= 0.0 || E.e2 <= prm.huber_delta * prm.huber_delta;
            wf_n[o] = inl ? 1 : 0;
            const double dr = (prm.huber_delta > 0.0) ? E.rho1 : 1.0;
            if (__ballot(!inl) == 0ull) lin_blocks<true>(E, pfixed, dr, hll, bl, hpl, trow);   // wave-uniform
            else lin_blocks<false>(E, pfixed, dr, hll, bl, hpl, trow);
        }
        STAMP(1);

        // ---- per-landmark H_ll, b_l over the lane group; Cholesky (redundant per lane) ----
        double h[9] = {hll[0], hll[1], hll[2], hll[3], hll[4], hll[5], bl[0], bl[1], bl[2]};
        group_sum(h, lg);
        // Cholesky of H_ll through reciprocal square roots: i_jj = 1/L_jj directly
        double i00 = fast_rsq(h[0]);
        const double l10 = h[1] * i00, l20 = h[2] * i00;
        const double a11 = h[3] - l10 * l10;
        const double i11 = fast_rsq(a11);
        const double l21 = (h[4] - l20 * l10) * i11;
        const double a22 = h[5] - l20 * l20 - l21 * l21;
        const double i22 = fast_rsq(a22);
        const bool pd = (h[0] > 0.0) && (a11 > 0.0) && (a22 > 0.0) && isfinite(i22) && isfinite(l21);
        // A landmark with one edge has a rank-2 H_ll: the reference's LU inverse (problem.cpp:399)
        // returns inf or rounding garbage for it.  Such a landmark (or a non-PD H_ll) poisons the
        // step like the inf does (guard 0: every trial is rejected, as the reference's solve is), or
        // is held fixed (guard 1).  The NaN reciprocal is the record's marker in both modes.
        const uint64_t vmask = __ballot(has);
        const uint64_t gmask = (lg >= 6) ? ~0ull : (((1ull << (1 << lg)) - 1ull) << (lane & ~((1 << lg) - 1)));
        const bool deg = !pd || __popcll(vmask & gmask) < 2;
        if (deg) i00 = __builtin_nan("");
        const double w0 = h[6] * i00, w1 = (h[7] - l10 * w0) * i11, w2 = (h[8] - l20 * w0 - l21 * w1) * i22;
        if (lead) {
            maxd = fmax(maxd, fmax(fabs(h[0]), fmax(fabs(h[3]), fabs(h[5]))));
            if (deg) ndeg += 1.0;
        }
        if (lmok) {
            // the record's eight 16-byte pieces from the landmark's lanes (every lane of the group holds the
            // same bits: butterfly totals, then the same arithmetic), piece q by lane q mod G: with G = 8 the
            // wave writes its 8 records as one contiguous 1 KB store (one piece per lane), whole 128-B lines
            // through the write-through path (8 pieces from the lead lane were 8 partial-line writes)
            double2* r2 = reinterpret_cast<double2*>(rn + ((size_t)sb * LH_SB_LM + ls) * LH_REC);
            for (int q = gj; q < 8; q += 1 << lg) {
                // piece q by a select tree on its bits (no divergent branches): 0 {X0, X1}, 1 {X2, i00},
                // 2 {l10, i11}, 3 {l20, l21}, 4 {i22, b0}, 5 {b1, b2}, 6 {H00, H11}, 7 {H22, 0}
                const bool q0 = q & 1, q1 = q & 2, q2 = q & 4;
                const double x01 = q0 ? X[2] : X[0], x23 = q0 ? l20 : l10, x45 = q0 ? h[7] : i22, x67 = q0 ? h[5] : h[0];
                const double y01 = q0 ? i00 : X[1], y23 = q0 ? l21 : i11, y45 = q0 ? h[8] : h[6], y67 = q0 ? 0.0 : h[3];
                const double x03 = q1 ? x23 : x01, x47 = q1 ? x67 : x45, y03 = q1 ? y23 : y01, y47 = q1 ? y67 : y45;
                st_rec2(r2 + q, double2{q2 ? x47 : x03, q2 ? y47 : y03}, rec_rsrc, rec);
            }
        }
        STAMP(2);

        // ---- per observation: G = H_pl L^-T and bsd = G w = H_pl H_ll^-1 b_l ----
        double G[18];
#pragma unroll
        for (int i = 0; i < 18; ++i) G[i] = 0.0;
        const bool gl = live && !(prm.guard && deg);
        if (gl) {
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                const double g0 = hpl[3 * a] * i00;
                const double g1 = (hpl[3 * a + 1] - l10 * g0) * i11;
                const double g2 = (hpl[3 * a + 2] - l20 * g0 - l21 * g1) * i22;
                G[3 * a] = g0; G[3 * a + 1] = g1; G[3 * a + 2] = g2;
                trow[27 + a] = g0 * w0 + g1 * w1 + g2 * w2;
            }
        }
        STAMP(3);

        // ---- per-pose sums (H_pp, b_p, bsd): the owner of cell (slot, task) adds it over every
        //      landmark observing the slot, in landmark (= lane) order ----
        wave_sync();
        {
            // every (landmark, slot) cell in landmark order: absent cells are +0.0, and adding
            // them leaves every sum bit-identical to adding the present cells only.  Cell c of
            // landmark l sits at scr[l * UMAX * 33 + c]: a wave's reads are contiguous.
#pragma unroll
            for (int i = 0; i < NCELL; ++i) {
                const int c = lane + 64 * i;
                if (c < U * LH_TASKS) {
                    double tv[LH_SB_LM];
#pragma unroll
                    for (int l = 0; l < LH_SB_LM; ++l) tv[l] = scr[l * Cfg::UMAX * LH_TASKS + c];
                    double sacc = task[i];
#pragma unroll
                    for (int l = 0; l < LH_SB_LM; ++l) sacc += tv[l];
                    task[i] = sacc;
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
    {   // the wave's totals: DPP and permlane butterflies (no LDS round trips); max |diag H_ll| likewise
        double t3[3] = {chi_acc, scale_acc, ndeg};
        group_sum(t3, 6);
        chi_acc = t3[0]; scale_acc = t3[1]; ndeg = t3[2];
        maxd = wave_max(maxd);
    }
    STAMP(9);
    lds_barrier();
    STAMP(8);
    double* smem = dsm;
    if (evo) {   // the chunk's scalars only, combined in the same order as below
        for (int phase = 0; phase < 2; ++phase) {
            if ((wave >> 1) == phase && lane == 0) {
                double* sc = smem + (wave & 1) * 2;
                if (phase == 0) { sc[0] = chi_acc; sc[1] = scale_acc; }
                else { sc[0] += chi_acc; sc[1] += scale_acc; }
            }
            lds_barrier();
        }
        double* gs = csc + (size_t)chunk * 4;
        if (tid < 2) gs[tid] = smem[tid] + smem[2 + tid];
        if (tid == 2 || tid == 3) gs[tid] = 0.0;
        return;
    }
    for (int phase = 0; phase < 2; ++phase) {
        if ((wave >> 1) == phase) {
            double* sl = smem + (wave & 1) * Cfg::LS;
            const bool first = phase == 0;
#pragma unroll
            for (int t = 0; t < Cfg::NT; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int idx = t * 256 + ((lane >> 4) + 4 * i) * 16 + (lane & 15);
                    sl[idx] = (first ? 0.0 : sl[idx]) + acc[t][i];
                }
#pragma unroll
            for (int i = 0; i < NCELL; ++i) {
                const int c = lane + 64 * i;
                if (c < U * LH_TASKS) {
                    const int idx = Cfg::LS_TASK + c;
                    sl[idx] = (first ? 0.0 : sl[idx]) + task[i];
                }
            }
            if (lane == 0) {
                double* sc = sl + Cfg::LS_SC;
                if (first) { sc[0] = chi_acc; sc[1] = scale_acc; sc[2] = ndeg; sc[3] = maxd; }
                else { sc[0] += chi_acc; sc[1] += scale_acc; sc[2] += ndeg; sc[3] = fmax(sc[3], maxd); }
            }
        }
        lds_barrier();
    }
    STAMP(9);
    // the chunk's contribution to each pose pair of its window, one pair row each (pair-major,
    // rows of one pair contiguous: k_reduce's loads need no index word).  Row: [0, 36) the
    // landmark part of S block (p, q), row-major; diagonal pairs also [36, 69) the pose's 33 sums.
    const double* s0 = smem;
    const double* s1 = smem + Cfg::LS;
    const uint32_t* wrow = reinterpret_cast<const uint32_t*>(wext + ncam * LH_EXT);
    {
        const int a = lane / 6, bb = lane - 6 * (lane / 6);
        int lp = 0;
        for (int s = 0; s < U; ++s)
            for (int t = s; t < U; ++t, ++lp) {
                if ((lp & (LH_WAVES - 1)) != wave) continue;
                double* row = rows + (size_t)wrow[lp] * LH_ROW;
                if (lane < 36) {
                    int ra = 6 * s + a, rc = 6 * t + bb;
                    if ((ra >> 4) > (rc >> 4)) { const int x = ra; ra = rc; rc = x; }
                    const int R = ra >> 4, Cc = rc >> 4;
                    const int idx = (R * T - (R * (R - 1)) / 2 + (Cc - R)) * 256 + (ra & 15) * 16 + (rc & 15);
                    st_out(row + lane, s0[idx] + s1[idx]);
                }
                if (s == t && lane < LH_TASKS)
                    st_out(row + 36 + lane, s0[Cfg::LS_TASK + s * LH_TASKS + lane] + s1[Cfg::LS_TASK + s * LH_TASKS + lane]);
            }
    }
    double* gs = csc + (size_t)chunk * 4;
    if (tid < 3) gs[tid] = s0[Cfg::LS_SC + tid] + s1[Cfg::LS_SC + tid];
    if (tid == 3) gs[3] = fmax(s0[Cfg::LS_SC + 3], s1[Cfg::LS_SC + 3]);
    STAMP(10);
    STAMP_FLUSH(0, 11);
}

// ============================================================================
// LM bookkeeping shared by the controllers (isGoodStepInLM, computeLambdaInitLM)
// ============================================================================
struct CtrlWords {
    double chi, lam, ni, last, spose, chi0;
    int iter, fc, trials, nacc, done, cur, tl;
    int evo, relin;   // this trial only evaluated; this chain re-linearises (the previous trial was such an acceptance)
    int retrial;      // this chain re-runs a batch's accepted rung (lh_ctrl.retrial: 2 when that acceptance stopped the loop)
    int lad, lad_n;   // the rung this trial's step came from; the rungs built (lh_ctrl.lad)
};
__device__ __forceinline__ CtrlWords ctrl_load(const lh_ctrl* __restrict__ ctrl) {
    CtrlWords w;
    w.chi = ctrl->chi; w.lam = ctrl->lambda; w.ni = ctrl->ni; w.last = ctrl->last_chi;
    w.chi0 = ctrl->chi2_initial;
    w.iter = ctrl->iter; w.fc = ctrl->false_cnt; w.trials = ctrl->trials; w.nacc = ctrl->accepted;
    w.done = ctrl->done; w.cur = ctrl->cur; w.tl = ctrl->trace_len;
    w.evo = ctrl->evo; w.relin = ctrl->relin; w.retrial = ctrl->retrial;
    w.lad = ctrl->lad; w.lad_n = ctrl->lad_n;
    // every rung's gain part is loaded and the trial's selected (no load that waits on lad)
    double sp[LH_LAD];
#pragma unroll
    for (int i = 0; i < LH_LAD; ++i) sp[i] = ctrl->spose_l[i];
    w.spose = sp[0];
#pragma unroll
    for (int i = 1; i < LH_LAD; ++i) w.spose = (w.lad == i) ? sp[i] : w.spose;
    return w;
}
// A batch's decisions (k_reduce) run back to back on one thread: the controller words and the
// counters they update stay in registers between the rungs, the rungs' gain parts and PCG counts in LDS (reloading
// them from lh_ctrl after each decision cost two dependent round trips per rung); each decision still stores its
// words.
struct BatchWords {
    CtrlWords w;              // the words the next rung's decision starts from
    const double* sp;         // lh_ctrl.spose_l (an LDS copy)
    const int* lad_its;       // lh_ctrl.lad_its (an LDS copy)
    int* cnt;                 // (LDS) lh_ctrl's counters lskips, pcg_iters; the last decision's lskip
};
enum { BW_LSKIPS, BW_PCG, BW_LSKIP };
__device__ __forceinline__ void batch_load(const lh_ctrl* __restrict__ ctrl, BatchWords& b, double* sp, int* its, int* cnt) {
    b.w = ctrl_load(ctrl);
#pragma unroll
    for (int i = 0; i < LH_LAD; ++i) { sp[i] = ctrl->spose_l[i]; its[i] = ctrl->lad_its[i]; }
    b.sp = sp;
    b.lad_its = its;
    b.cnt = cnt;
    cnt[BW_LSKIPS] = ctrl->lskips;
    cnt[BW_PCG] = ctrl->pcg_iters;
    cnt[BW_LSKIP] = 0;
}

// a batch's words after its last decision (what ctrl_lm_step stores after a decision, from the batch's registers)
__device__ __forceinline__ void batch_store(lh_ctrl* __restrict__ ctrl, const BatchWords& b, int seq) {
    const CtrlWords& o = b.w;
    ctrl->chi = o.chi; ctrl->lambda = o.lam; ctrl->ni = o.ni; ctrl->last_chi = o.last; ctrl->chi2_initial = o.chi0;
    ctrl->iter = o.iter; ctrl->false_cnt = o.fc; ctrl->trials = o.trials; ctrl->accepted = o.nacc;
    ctrl->done = o.done; ctrl->cur = o.cur; ctrl->trace_len = o.tl;
    ctrl->retrial = o.retrial;
    ctrl->lad = o.lad;
    ctrl->lskip = b.cnt[BW_LSKIP];
    ctrl->lskips = b.cnt[BW_LSKIPS];
    ctrl->pcg_iters = b.cnt[BW_PCG];
    ctrl->acc_hist[seq & 1] = 0;   // a batch commits nothing (a retrial does)
    ctrl->seq_last = seq;
    ctrl->relin = o.relin;
    ctrl->nofactor = o.relin | b.cnt[BW_LSKIP] | (o.retrial != 0 ? 1 : 0);
    ctrl->evo = o.evo;
    ctrl->evo_seq[(seq + 1) & 1] = o.evo;
}

// The stop trial's summary and trace to the host words, then done, by ONE thread behind its own
// system-scope fence.  A kernel boundary releases at agent scope only, and the trace entries were
// decided by earlier kernels on other CUs, so every word the host reads after done is stored here,
// from lh_ctrl (device memory, complete at this kernel's start or written by this thread).  The words
// are plain stores, issued back to back, and the one fence orders them all before done (volatile
// stores each waited for their own write to the host: the stop's controller took ~18 us).
__device__ __noinline__ void publish_stop(const lh_ctrl* __restrict__ ctrl, volatile int* __restrict__ host_done) {
    lh_host_words* hw = reinterpret_cast<lh_host_words*>(const_cast<int*>(host_done));
    const int tl = ctrl->trace_len, nt = tl < LH_TRACE ? tl : LH_TRACE;
    hw->iter = ctrl->iter; hw->trials = ctrl->trials; hw->accepted = ctrl->accepted; hw->trace_len = tl;
    hw->nonpd = ctrl->nonpd; hw->pcg_iters = ctrl->pcg_iters;
    hw->chi2_initial = ctrl->chi2_initial; hw->chi = ctrl->chi; hw->lambda = ctrl->lambda;
    // four entries' loads in flight (unconditional, in the array), then their stores: few registers, so that a
    // caller's live values need no saving around this call (sixteen at a time spilled k_ctrl<0, false>)
    for (int i0 = 0; i0 < nt; i0 += 4) {
        double c[4], l[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = min(i0 + j, LH_TRACE - 1);
            c[j] = ctrl->trace_chi[i];
            l[j] = ctrl->trace_lambda[i];
        }
        // (unconditional too: an entry past trace_len is never read by the host, and a store behind a branch
        // waited for the stores before it)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = min(i0 + j, LH_TRACE - 1);
            hw->trace_chi[i] = c[j];
            hw->trace_lambda[i] = l[j];
        }
    }
    __threadfence_system();
    host_done[0] = 1;
}

// The host's progress word after chain seq's decision (ctrl_lm_step; a batch's after its last rung, k_reduce):
// 2 seq + near, near = 1 when the next chain may be the last (one more completed iteration reaches max_iters, a
// stalled iteration's last rejection, or a pending retrial that stops the loop).
__device__ __forceinline__ void ctrl_progress(const lh_params& prm, volatile int* __restrict__ host_done, int seq, int iter,
                                              int fc, double last, double chi, int hold) {
    const int near = (prm.max_iters > 0 && iter + 1 >= prm.max_iters) ? 1 : 0;
    const int last_try = (fc + 1 >= prm.max_trials && last - chi < prm.stop_dchi2) ? 1 : 0;
    host_done[1] = 2 * seq + (near | last_try | hold);
}

// Returns 1 when the controller has nothing to factor: this trial was an evaluate-only one accepted outside the
// final iteration (the next chain re-linearises the accepted state, relin; that chain's decision commits the new
// linearisation like the initial one and leaves the LM state alone), a rejection whose step a lambda-ladder
// rung already holds (lskip), or a batch's acceptance (retrial).
// batch: the decision of one rung of a batch (k_reduce's loop over the rungs a chain evaluated):
// an acceptance commits nothing (the next chain re-runs the rung as a full trial, lh_ctrl.retrial, and its
// decision commits it; a stop it causes is raised by that chain), and the host word is the loop's to write.
__device__ __forceinline__ int ctrl_lm_step(lh_ctrl* __restrict__ ctrl, const CtrlWords& w, const lh_params& prm,
                                             int mode, double mdiag, double tchi, double sl, double ndg,
                                             volatile int* __restrict__ host_done, int seq, int& done_o, int& accept_o,
                                             int& cur_o, double& lam_o, bool raise_done = true, BatchWords* bw = nullptr,
                                             bool in_batch = true) {
    // (bw is always a valid pointer where the decision may be a batch's, and in_batch says whether it is one: a
    // pointer chosen at run time would keep the caller's words out of registers)
    const bool batch = bw != nullptr && in_batch;
    double chi = w.chi, lam = w.lam, ni = w.ni, last = w.last, spose = w.spose, chi0 = w.chi0;
    int iter = w.iter, fc = w.fc, trials = w.trials, nacc = w.nacc, tl = w.tl;
    int done = w.done, cur = w.cur;
    int accept = 0, trace = 0, relin = 0, retrial = 0;
    int lad = 0, lskip = 0;   // the next step's rung: 0 after any factor; a rejection moves up the ladder
    if (!done) {
        if (mode != 0 && (w.relin || w.retrial)) {
            // the re-linearisation of an evaluate-only acceptance: its records and pose tables were written
            // to the candidate side (k_lin), which becomes the committed one; lambda, chi2 and the counts
            // were updated by the acceptance.  A retrial (a batch's accepted rung as a full trial) likewise,
            // and it raises the stop that acceptance took.
            cur = 1 - cur;
            accept = 1;
            if (w.retrial == 2) done = 1;
        } else if (mode == 0) {
            // computeLambdaInitLM (problem.cpp:470-504)
            ni = 2.0;
            chi = tchi;
            chi0 = tchi;
            if (prm.strategy == 0) {
                if (!prm.lambda_given) {
                    double m = fmin(prm.lambda_cap, mdiag);
                    lam = prm.tau * m;
                } else {
                    lam = prm.lambda_init;
                }
            } else {
                lam = 1e-5;
            }
            last = 1e20;
            iter = 0; fc = 0; trials = 0; nacc = 0; tl = 0;
            ctrl->nonpd = (int)ndg;
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
                    const double m = 2 * rho - 1;
                    double alpha = 1.0 - m * m * m;   // std::pow(2 rho - 1, 3), problem.cpp:541 (within an ulp)
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
                if (!batch) {
                    cur = 1 - cur;   // commit candidate landmarks, caches and poses
                    accept = 1;
                } else {
                    retrial = 1;     // the next chain linearises this rung's candidate (its step: rung w.lad)
                    lad = w.lad;
                }
                fc = 0;
                inner_end = true;
            } else {
                fc += 1;             // rollbackStates: the committed buffers are untouched
                inner_end = fc >= prm.max_trials;
                // the lambda just set is the next rung's (the ladder applied the same updates in the same order):
                // its step is already solved, so this chain's controller has nothing to factor
                if (w.lad + 1 < w.lad_n) {
                    lad = w.lad + 1;
                    lskip = 1;
                }
            }
            relin = (ok && w.evo && !batch) ? 1 : 0;   // (cleared below when the loop stops)
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
        if (retrial && done) retrial = 2;   // the stop is the retrial's to raise
        if (done) lskip = 0;
        if (done) relin = 0;
        // (a batch's rung stores its words once, after the batch's last decision: batch_store)
        if (!batch) {
            ctrl->chi = chi; ctrl->lambda = lam; ctrl->ni = ni; ctrl->last_chi = last; ctrl->chi2_initial = chi0;
            ctrl->iter = iter; ctrl->false_cnt = fc; ctrl->trials = trials; ctrl->accepted = nacc;
            ctrl->done = retrial ? 0 : done; ctrl->cur = cur; ctrl->trace_len = tl;
            ctrl->retrial = retrial;
            ctrl->rho_sel = 0;
            ctrl->lad = lad;
            ctrl->lskip = lskip;
            if (lskip) ctrl->lskips += 1;
            if (lskip && prm.solver == 1) ctrl->pcg_iters += ctrl->lad_its[lad];   // the rung's solve counts now
            ctrl->acc_hist[seq & 1] = accept;
            ctrl->seq_last = seq;
            ctrl->relin = relin;
            ctrl->nofactor = relin | lskip | (retrial != 0 ? 1 : 0);
        } else {   // (the same counts from the batch's registers)
            bw->cnt[BW_LSKIPS] += lskip;
            if (lskip && prm.solver == 1) bw->cnt[BW_PCG] += bw->lad_its[lad];
        }
        // The next trial is in the final iteration when one more completed iteration reaches max_iters.
        // Its decision then either stops the loop (accept, or the last rejection) or leads to another
        // such trial, so its candidate linearisation is never used: k_lin only evaluates (evo).  With
        // prm.eval_first a trial after a rejection in its iteration also only evaluates: a run of
        // rejections (every solve that stops on a stalled chi2 ends with max_trials of them) then pays
        // evaluations only, and an acceptance among them one re-linearisation chain (relin).
        const int near = (prm.max_iters > 0 && iter + 1 >= prm.max_iters) ? 1 : 0;
        // A retrial is a full trial (it linearises the accepted rung's candidate, as a re-linearisation does), or an
        // evaluate-only one when that acceptance stopped the loop (it then only writes the candidate, as the serial
        // evaluate-only trial that stopped the loop did)
        const int evo_n = retrial == 2 ? 1
                        : (done || relin || retrial || prm.no_evo) ? 0 : (near | ((prm.eval_first && fc > 0) ? 1 : 0));
        // the next chain evaluates a batch of rungs when it is an evaluate-only trial after a rejection onto a built
        // rung: the rungs from there up to the last built one, within the trials left in the iteration
        const int nbatch_n = (prm.batch > 1 && evo_n && fc > 0 && lskip) ? min(min(w.lad_n - lad, prm.max_trials - fc), prm.batch) : 1;
        // (the evo words: evo in the low byte, a batch's rung count above it)
        const int evw = evo_n | (nbatch_n > 1 ? nbatch_n << 8 : 0);
        if (!batch) {
            ctrl->evo = evw;
            ctrl->evo_seq[(seq + 1) & 1] = evw;
        }
        // host words: [0] the loop stopped; else [1] = 2 seq + near, the progress word: this live
        // trial's controller has decided (its k_lin and k_reduce are done), and near = 1 when one
        // more completed iteration reaches max_iters.  The host keeps the queue filled from it (one
        // trial ahead when near, so a stop by max_iters leaves nothing enqueued past it); it never
        // advances past the stop trial, which bounds how many trials (and all-reduces) any rank
        // can have enqueued.  One 32-bit store: the host never sees a torn pair.
        if (host_done && !batch) {
            if (done) {
                ctrl->done_seq = seq;
                if (raise_done) publish_stop(ctrl, host_done);   // reads back this thread's stores above
                // else the same trial's controller publishes the summary from lh_ctrl and raises done
                // (publish_stop): only stores of the thread that fences are ordered before done
            } else {
                // near also when the next trial's rejection would end its iteration at an unchanged chi2 (a
                // stalled solve's last trial: the stop rule then ends the loop), so no chain is left past it; and
                // likewise when the next chain is a batch whose last rung is such a trial
                const int hold = (nbatch_n > 1 && fc + nbatch_n >= prm.max_trials && last - chi < prm.stop_dchi2) ? 1 : 0;
                ctrl_progress(prm, host_done, seq, iter, fc, last, chi, hold);
            }
        }
        if (retrial == 2) done = 0;
        if (batch) {   // the words the next rung's decision starts from (as ctrl_load would read them back)
            CtrlWords& o = bw->w;
            o.chi = chi; o.lam = lam; o.ni = ni; o.last = last; o.chi0 = chi0;
            o.iter = iter; o.fc = fc; o.trials = trials; o.nacc = nacc; o.done = done; o.cur = cur; o.tl = tl;
            o.evo = evw; o.relin = relin; o.retrial = retrial; o.lad = lad;
            o.spose = bw->sp[lad];
            bw->cnt[BW_LSKIP] = lskip;
        }
    }
    done_o = done;
    accept_o = accept;
    cur_o = cur;
    lam_o = lam;
    // nothing to factor: an evaluate-only acceptance, a rejection onto a built rung, or a batch's acceptance
    return relin | lskip | (retrial != 0 ? 1 : 0);
}

// A batch's decisions, thread 0 of the deciding kernel (k_reduce with one rank, else the
// controller after the exchange): rung r's chi2 (not halved) and gain scale at sc[2 r], sc[2 r + 1] (summed over
// the chunks, and over the ranks when sharded, as a single trial's are), decided in order until an acceptance
// (retrial), the stop, or a next trial that is not the batch's next rung.  bw holds the words batch_load read.
//
// (1) The rungs before the first that will be accepted (or the last) are plain rejections: each only advances
// lambda and nu, the counts and the rung (ctrl_lm_step's rejection, which moves onto a built rung and, before the
// batch's last rung, never ends the iteration: nbatch <= max_trials - false_cnt).  Their gain ratios are
// independent (chi2 does not change across rejections), so they are found first and skipped forward with that
// arithmetic; ctrl_lm_step takes the decisive rung.  Returns that rung.
__device__ __forceinline__ int batch_skip_forward(BatchWords& bw, const lh_params& prm, const double* sc, int nb) {
    CtrlWords& w = bw.w;
    const double chi = w.chi;
    int j = nb - 1;
    for (int q = 0; q < nb - 1; ++q) {
        double scale = 0.5 * (bw.sp[w.lad + q] + sc[2 * q + 1]);
        scale += 1e-10;
        const double tchi = 0.5 * sc[2 * q];
        const double rho = (chi - tchi) / scale;
        if (rho > 0 && isfinite(tchi)) { j = q; break; }
    }
    for (int r = 0; r < j; ++r) {   // rung r rejected: the decision ctrl_lm_step takes for it, in its order
        if (prm.strategy == 0) { w.lam *= w.ni; w.ni *= 2; }
        else w.lam = fmin(w.lam * 11.0, 1e7);
        w.trials += 1;
        w.fc += 1;
        w.lad += 1;
        bw.cnt[BW_LSKIPS] += 1;
        if (prm.solver == 1) bw.cnt[BW_PCG] += bw.lad_its[w.lad];
    }
    w.spose = bw.sp[w.lad];
    if (j > 0) bw.cnt[BW_LSKIP] = 1;
    return j;
}
// (2) after the decisive rung r: the words stored once, the rung whose rho0 is "as last evaluated", and the host word
// (raise_done: publish the stop here, else the chain's controller does).  Returns nothing-to-factor, with
// ctrl_lm_step's outputs.
__device__ __forceinline__ int batch_finish(lh_ctrl* __restrict__ ctrl, BatchWords& bw, const lh_params& prm, int r,
                                            volatile int* __restrict__ host_done, int seq, bool raise_done, int& done_o,
                                            int& accept_o, int& cur_o, double& lam_o) {
    const CtrlWords& w = bw.w;
    batch_store(ctrl, bw, seq);
    ctrl->rho_sel = r;   // the per-edge rho0 of the last rung decided
    ctrl->nbatches += 1;
    if (w.retrial) ctrl->nretrials[w.retrial - 1] += 1;
    if (host_done) {
        if (w.done) {
            ctrl->done_seq = seq;
            if (raise_done) publish_stop(ctrl, host_done);   // else this chain's controller publishes it
        } else {
            ctrl_progress(prm, host_done, seq, w.iter, w.fc, w.last, w.chi, w.retrial == 2 ? 1 : 0);
        }
    }
    done_o = w.done;
    accept_o = 0;
    cur_o = w.cur;
    lam_o = w.lam;
    return w.relin | bw.cnt[BW_LSKIP] | (w.retrial != 0 ? 1 : 0);
}
__device__ __forceinline__ bool batch_more(const BatchWords& bw, int r, int nb) {
    const CtrlWords& w = bw.w;
    return !(r + 1 >= nb || w.done || w.retrial || !w.evo || !bw.cnt[BW_LSKIP]);
}
// k_reduce's (one rank)
__device__ __forceinline__ int ctrl_batch_decide(lh_ctrl* __restrict__ ctrl, BatchWords& bw, const lh_params& prm,
                                                 const double* sc, int nb, volatile int* __restrict__ host_done, int seq,
                                                 bool raise_done, int& done_o, int& accept_o, int& cur_o, double& lam_o) {
    int r = batch_skip_forward(bw, prm, sc, nb);
    for (;; ++r) {
        int d_o, a_o, c_o;
        double l_o;
        ctrl_lm_step(ctrl, bw.w, prm, 1, 0.0, 0.5 * sc[2 * r], sc[2 * r + 1], 0.0, host_done, seq, d_o, a_o, c_o, l_o,
                     false, &bw);
        if (!batch_more(bw, r, nb)) break;
    }
    return batch_finish(ctrl, bw, prm, r, host_done, seq, raise_done, done_o, accept_o, cur_o, lam_o);
}
// a self-deciding controller's decision (thread 0): a batch's (this chain's evo word above its low byte, the
// rungs' scalars behind the exchanged system, lh_rs_layout.off_bsc) or one trial's.  BATCH false: the caller's
// batches are decided elsewhere (k_ctrl: its decider workgroup, ctrl_batch_decider)
template <bool BATCH = true>
__device__ __forceinline__ int ctrl_decide(lh_ctrl* __restrict__ ctrl, const CtrlWords& cw, const lh_params& prm, int mode,
                                           double mdiag, double tchi, double sl, double ndg, const double* rs_stage,
                                           const lh_rs_layout& LY, volatile int* __restrict__ host_done, int seq,
                                           int& done_o, int& accept_o, int& cur_o, double& lam_o, int* cnt) {
    if constexpr (BATCH) {
        const int nb = cw.evo >> 8;   // (cw.evo: this chain's evo word, read before its decision)
        if (mode != 0 && nb > 1) {
            BatchWords bw;
            bw.w = cw;
            bw.sp = ctrl->spose_l;   // (global: one load per rung)
            bw.lad_its = ctrl->lad_its;
            bw.cnt = cnt;
            cnt[BW_LSKIPS] = ctrl->lskips;
            cnt[BW_PCG] = ctrl->pcg_iters;
            cnt[BW_LSKIP] = 0;
            return ctrl_batch_decide(ctrl, bw, prm, rs_stage + LY.off_bsc, nb, host_done, seq, true, done_o, accept_o,
                                     cur_o, lam_o);
        }
    }
    return ctrl_lm_step(ctrl, cw, prm, mode, mdiag, tchi, sl, ndg, host_done, seq, done_o, accept_o, cur_o, lam_o);
}
// ---- the lambda ladder's rung workgroups (lh_ctrl.lad) ----
// Workgroup 0 of a controller that takes the LM decision itself (the initial linearisation, sharded solves,
// k_ctrl_g, k_ctrl_p) publishes it: ctrl_lm_step's words, then dec_tag = seq + 1 (release).  Its rung workgroups
// wait for that tag (acquire) and read the decision from lh_ctrl like a controller after k_reduce's decision.
// Workgroups are dispatched in order, so workgroup 0 is resident whatever the rungs do: the wait ends.
__device__ __forceinline__ void ladder_publish(lh_ctrl* __restrict__ ctrl, int seq) {
    __hip_atomic_store(&ctrl->dec_tag, seq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ladder_wait(const lh_ctrl* __restrict__ ctrl, int seq) {
    if (threadIdx.x == 0)
        while (__hip_atomic_load(&ctrl->dec_tag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != seq + 1)
            __builtin_amdgcn_s_sleep(2);
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // every wave's loads below see workgroup 0's words
}
// the decision as a rung reads it, and the rung's lambda: the updates `rung` more rejections apply to lambda and
// ni, in ctrl_lm_step's order (DEFAULT problem.cpp:550-551, STRATEGY1 :576), so each is bit-identical
struct LadderDec {
    int done, accept, skip;
    double lambda;
};
__device__ __forceinline__ LadderDec ladder_read(const lh_ctrl* __restrict__ ctrl, const lh_params& prm, int seq, int rung) {
    LadderDec d;
    d.done = __builtin_amdgcn_readfirstlane(ctrl->done);
    d.accept = __builtin_amdgcn_readfirstlane(ctrl->acc_hist[seq & 1]);
    // an evaluate-only acceptance (nothing to factor), or a rejection onto a built rung (its step is solved)
    d.skip = __builtin_amdgcn_readfirstlane(ctrl->nofactor);
    double lambda = ctrl->lambda, ni = ctrl->ni;
    for (int i = 0; i < rung; ++i) {
        if (prm.strategy == 0) { lambda *= ni; ni *= 2; }
        else lambda = fmin(lambda * 11.0, 1e7);
    }
    d.lambda = lambda;
    return d;
}
// k_ctrl's decider workgroup (the launch's last, when the controller decides itself: sharded solves): thread 0
// takes the chain's LM decision -- one trial's, or a batch's -- then publishes the tag the factoring workgroup and
// the rungs wait for (ladder_publish).  It holds no prefetched system: workgroup 0, deciding with that system in
// registers, spilled (k_ctrl<0, false>, once the decision learnt batches).
__device__ __forceinline__ void ctrl_decider(lh_ctrl* __restrict__ ctrl, const lh_params& prm, const double* rs_stage,
                                             const lh_rs_layout& LY, int nb, volatile int* __restrict__ host_done,
                                             int seq) {
    __shared__ int cnt[4];
    int d_o, a_o, c_o;
    double l_o;
    if (nb > 1) {
        BatchWords bw;
        bw.w = ctrl_load(ctrl);
        bw.sp = ctrl->spose_l;
        bw.lad_its = ctrl->lad_its;
        bw.cnt = cnt;
        cnt[BW_LSKIPS] = ctrl->lskips;
        cnt[BW_PCG] = ctrl->pcg_iters;
        cnt[BW_LSKIP] = 0;
        ctrl_batch_decide(ctrl, bw, prm, rs_stage + LY.off_bsc, nb, host_done, seq, true, d_o, a_o, c_o, l_o);
    } else {
        const CtrlWords cw = ctrl_load(ctrl);
        ctrl_lm_step(ctrl, cw, prm, 1, 0.0, 0.5 * rs_stage[LY.off_sc + LH_SC_CHI2], rs_stage[LY.off_sc + LH_SC_SCALE],
                     rs_stage[LY.off_sc + LH_SC_NDEG], host_done, seq, d_o, a_o, c_o, l_o);
    }
    ladder_publish(ctrl, seq);
}

// a factoring controller's rung count: prm.ladder rungs at every factor (ladder_eager) or a factor after a rejection
__device__ __forceinline__ bool ladder_build(const lh_params& prm, int accept) {
    return prm.ladder > 1 && (prm.ladder_eager || !accept);
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

// With prm.dec_in_reduce (one rank, P <= LH_PMAX) the scalar block also takes the trial's LM decision
// (isGoodStepInLM on its chi2 and gain-scale sums, the controller update, the host words): k_ctrl
// then reads accept / lambda with its prefetch instead of deciding on one thread behind it.
// With prm.commit_in_reduce each pair block first copies its staged entries to the committed system
// when the previous trial was accepted (before this trial overwrites them; an evaluate-only trial
// copies and writes nothing): a controller that factors a large system then never copies it.
__global__ __launch_bounds__(RT) void k_reduce(const double* __restrict__ rows, const double* __restrict__ csc,
                                               const uint4* __restrict__ red_tab, int nred,
                                               lh_ctrl* __restrict__ ctrl, double* __restrict__ rs,
                                               double* __restrict__ rs_commit, double* __restrict__ maxd_out,
                                               lh_params prm, int n_chunks, int mode, volatile int* __restrict__ host_done,
                                               int seq, double* __restrict__ img) {
    STAMP_DECL
    __shared__ double part[3][RW][64];
    const lh_rs_layout LY = lh_rs_make(prm.P, prm.npairs);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // the stop flag and this block's pair words (one 16-byte entry of the host's table: the pairs some chunk
    // reaches, then the scalar block's sentinel {npairs, 0, 0, 0}) are independent loads: one round trip
    const uint4 rt = red_tab[min((int)blockIdx.x, nred)];
    const int b = (int)blockIdx.x < nred ? (int)rt.x : LY.npairs;
    const int ib = (int)rt.y, ie = (int)rt.z;
    const int p = (int)(rt.w & 0xffffu), q = (int)(rt.w >> 16);
    const int done = __builtin_amdgcn_readfirstlane(ctrl->done);
    // k_lin wrote the chunk scalars only (this trial's word: the scalar block's decision writes the next one's)
    // this chain's evo word (evo, and above it a batch's rung count: k_lin evaluated rungs lad .. lad + nb - 1, their
    // chunk scalars at csc + r n_chunks 4)
    const int evo = mode != 0 ? __builtin_amdgcn_readfirstlane(ctrl->evo_seq[seq & 1]) : 0;
    const int nb = max(evo >> 8, 1);
    const bool copy_prev = (prm.commit_in_reduce | prm.img) && mode != 0 && b < LY.npairs && done == 0 && wave == 0;
    const int prev_acc = copy_prev ? __builtin_amdgcn_readfirstlane(ctrl->acc_hist[(seq - 1) & 1]) : 0;
    if (copy_prev) {
        if (prev_acc) {
            if (prm.img) {   // this pair's entries of k_ctrl's image (their slots below), then the rhs row's
                if (lane < 36) {
                    const int ea_ = lane / 6, eb_ = lane - 6 * (lane / 6), gi = 6 * p + ea_, gj = 6 * q + eb_;
                    const int idx = (p < q) ? gj * LH_IMG_AS + gi : ((ea_ >= eb_) ? gi * LH_IMG_AS + gj : -1);
                    if (idx >= 0) st_red(img + LH_IMG_SZ + idx, img[idx]);
                } else if (p == q && lane < 42) {
                    const int idx = LH_NPAD * LH_IMG_AS + 6 * p + (lane - 36);
                    st_red(img + LH_IMG_SZ + idx, img[idx]);
                }
            } else if (prm.bimg) {   // this pair's entries of k_ctrl_b's band image
                const int bsz = ((6 * prm.P + 15) >> 4) * LH_BIMG_TR;
                if (lane < 36) {
                    const int ea_ = lane / 6, eb_ = lane - 6 * (lane / 6), gi = 6 * p + ea_, gj = 6 * q + eb_;
                    const int r_ = (p < q) ? gj : gi, c_ = (p < q) ? gi : gj;
                    if ((p < q || ea_ >= eb_) && lh_bimg_in(r_, c_)) st_red(img + bsz + lh_bimg_idx(r_, c_), img[lh_bimg_idx(r_, c_)]);
                }
            } else if (lane < 36) {
                st_red(rs_commit + LY.off_S + b * 36 + lane, rs[LY.off_S + b * 36 + lane]);
            }
            if (p == q && lane >= 36 && lane < 54) {
                const int k = lane - 36, part_off = (k < 6) ? LY.off_bs : (k < 12) ? LY.off_bp : LY.off_hd;
                const int i = part_off + 6 * p + (k % 6);
                st_red(rs_commit + i, rs[i]);
            }
        }
    }
    // An evaluate-only trial writes no system, and if it is rejected its controller factors the committed one:
    // k_ctrl's image path loads the staged image before the decision is known, so this pair's committed
    // entries (image slots, rhs row, b_s, b_p, diag H_pp) are copied to the staged side here, and that
    // controller then needs no second load after a rejection.  After an accepted trial the copy above has
    // just made the two sides equal, and this one is skipped.
    if (prm.img && evo && !prev_acc && b < LY.npairs && done == 0 && wave == 0) {
        if (lane < 36) {
            const int ea_ = lane / 6, eb_ = lane - 6 * (lane / 6), gi = 6 * p + ea_, gj = 6 * q + eb_;
            const int idx = (p < q) ? gj * LH_IMG_AS + gi : ((ea_ >= eb_) ? gi * LH_IMG_AS + gj : -1);
            if (idx >= 0) st_red(img + idx, img[LH_IMG_SZ + idx]);
        } else if (p == q && lane < 42) {
            const int idx = LH_NPAD * LH_IMG_AS + 6 * p + (lane - 36);
            st_red(img + idx, img[LH_IMG_SZ + idx]);
        }
        if (p == q && lane >= 36 && lane < 54) {
            const int k = lane - 36, part_off = (k < 6) ? LY.off_bs : (k < 12) ? LY.off_bp : LY.off_hd;
            const int i = part_off + 6 * p + (k % 6);
            st_red(rs + i, rs_commit[i]);
        }
    }
    // (p > q and ib > ie never hold: they make the exit test need the pair words, so the compiler issues
    // them with the controller's instead of sinking them below the branch, a second round trip)
    if ((done != 0) | ((evo != 0) & (b < LY.npairs)) | (p > q) | (ib > ie)) return;   // no short-circuit: one test
    if (b == LY.npairs) {
        // the LM decision's controller words go out with the chunk scalars (one round trip, not a third
        // after the sums; only this block's thread 0 writes them in this kernel)
        CtrlWords cw0{};
        BatchWords bw0;
        __shared__ double b_sp[LH_LAD];
        __shared__ int b_its[LH_LAD], b_cnt[4];
        if (prm.dec_in_reduce && mode != 0 && tid == 0) {
            if (nb > 1) batch_load(ctrl, bw0, b_sp, b_its, b_cnt);
            else cw0 = ctrl_load(ctrl);
        }
        if (nb > 1) {
            // each rung's chi2 and gain-scale sums in the order below (thread, lane butterfly, waves in order):
            // ten rungs (a default ladder's batch) per round of loads, the butterflies in VALU (wave_sum_desc)
            constexpr int BG = 10;
            for (int g = 0; g < nb; g += BG) {
                double b[2 * BG];
#pragma unroll
                for (int j = 0; j < 2 * BG; ++j) b[j] = 0.0;
                for (int c = tid; c < n_chunks; c += RT) {
#pragma unroll
                    for (int j = 0; j < BG; ++j)
                        if (g + j < nb) {
                            const double* sc = csc + ((size_t)(g + j) * n_chunks + c) * 4;
                            b[2 * j] += sc[0]; b[2 * j + 1] += sc[1];
                        }
                }
                wave_sum_desc(b);
                if (lane == 0)
#pragma unroll
                    for (int j = 0; j < 2 * BG; ++j)
                        if (2 * g + j < 2 * nb) part[0][wave][2 * g + j] = b[j];
            }
            lds_barrier();
            // each rung's totals over the waves, in wave order, by one thread per rung: into LDS for the decisions
            // here (one rank), and behind the system (off_bsc) for the exchange and a controller that decides
            __shared__ double b_a[2 * LH_LAD];
            if (tid < nb) {
                double a0 = 0.0, a1 = 0.0;
                for (int wv = 0; wv < RW; ++wv) { a0 += part[0][wv][2 * tid]; a1 += part[0][wv][2 * tid + 1]; }
                b_a[2 * tid] = a0;
                b_a[2 * tid + 1] = a1;
                rs[LY.off_bsc + 2 * tid] = a0;
                rs[LY.off_bsc + 2 * tid + 1] = a1;
            }
            if (tid == 0) {
                rs[LY.off_sc + LH_SC_CHI2] = 0.0; rs[LY.off_sc + LH_SC_SCALE] = 0.0;
                rs[LY.off_sc + LH_SC_NDEG] = 0.0; rs[LY.off_sc + LH_SC_MAXD] = 0.0;
                *maxd_out = 0.0;
            }
            lds_barrier();
            if (prm.dec_in_reduce && tid == 0) {
                int d_o, a_o, c_o;
                double l_o;
                ctrl_batch_decide(ctrl, bw0, prm, b_a, nb, host_done, seq, false, d_o, a_o, c_o, l_o);
            }
            return;
        }
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, mx = 0.0;
        for (int c = tid; c < n_chunks; c += RT) {
            const double* sc = csc + (size_t)c * 4;
            s0 += sc[0]; s1 += sc[1]; s2 += sc[2]; mx = fmax(mx, sc[3]);
        }
        for (int off = 32; off > 0; off >>= 1) {
            s0 += __shfl_xor(s0, off); s1 += __shfl_xor(s1, off); s2 += __shfl_xor(s2, off);
            mx = fmax(mx, __shfl_xor(mx, off));
        }
        if (lane == 0) { part[0][wave][0] = s0; part[1][wave][0] = s1; part[2][wave][0] = s2; part[0][wave][1] = mx; }
        lds_barrier();
        if (tid == 0) {
            double a0 = 0.0, a1 = 0.0, a2 = 0.0, m = 0.0;
            for (int w = 0; w < RW; ++w) { a0 += part[0][w][0]; a1 += part[1][w][0]; a2 += part[2][w][0]; m = fmax(m, part[0][w][1]); }
            rs[LY.off_sc + LH_SC_CHI2] = a0;
            rs[LY.off_sc + LH_SC_SCALE] = a1;
            rs[LY.off_sc + LH_SC_NDEG] = a2;
            rs[LY.off_sc + LH_SC_MAXD] = m;
            *maxd_out = m;
            if (prm.dec_in_reduce && mode != 0) {
                int d_o, a_o, c_o;
                double l_o;
                ctrl_lm_step(ctrl, cw0, prm, 1, 0.0, 0.5 * a0, a1, a2, host_done, seq, d_o, a_o, c_o, l_o, false);
            }
        }
        return;
    }
    const bool diag = p == q;
    const int a = lane / 6, bb = lane - 6 * (lane / 6);
    // lanes 0..35: S entry (a, bb) [+ H_pp entry on the diagonal]; 36..41: b_p; 42..47: bsd
    int off_h = 0;
    if (lane < 36) off_h = 36 + (diag ? hpp_index(a < bb ? a : bb, a < bb ? bb : a) : 0);
    else if (lane < 42) off_h = 36 + 21 + (lane - 36);
    else if (lane < 48) off_h = 36 + 27 + (lane - 42);
    const bool act_s = lane < 36, act_h = (lane < 36 && diag) || (lane >= 36 && lane < 48 && diag);
    // Each wave walks its rows (wave, wave + RW, ...) in order, eight at a time; the addresses
    // follow from the pair's row range alone, so every load of the pair is in flight together.
    double vs = 0.0, vh = 0.0;
    const int w_u = __builtin_amdgcn_readfirstlane(wave);
    // 24 rows per wave per round: a C3 diagonal pair's ~300 rows arrive in one round trip (8 took three:
    // 6.67 -> 6.44 us per launch; 16 took two and measured 7.2, its doubled loads per round slower)
    constexpr int LH_RED_ROWS = 24;
    for (int base = ib + w_u; base < ie; base += LH_RED_ROWS * RW) {
        double x[LH_RED_ROWS], y[LH_RED_ROWS];
#pragma unroll
        for (int u = 0; u < LH_RED_ROWS; ++u) {
            const int it = base + u * RW;
            const bool in = it < ie;
            const double* row = rows + (size_t)(in ? it : ib) * LH_ROW;
            x[u] = (in && act_s) ? row[lane] : 0.0;
            y[u] = (in && act_h) ? row[off_h] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < LH_RED_ROWS; ++u) { vs += x[u]; vh += y[u]; }
    }
    part[0][wave][lane] = vs;
    part[1][wave][lane] = vh;
    lds_barrier();
    if (wave == 0) {
        double s = 0.0, h = 0.0;
        for (int w = 0; w < RW; ++w) { s += part[0][w][lane]; h += part[1][w][lane]; }
        if (lane < 36) {
            const double v = (diag ? h : 0.0) - s;
            if (prm.img) {
                // k_ctrl's LDS layout (prm.img): entry (a, bb) of block (p, q) is S(6p + a, 6q + bb); its lower
                // slot only (the upper triangle stays zero in the image, where the factor writes L^T)
                const int gi = 6 * p + a, gj = 6 * q + bb;
                if (p < q) st_red(img + gj * LH_IMG_AS + gi, v);
                else if (a >= bb) st_red(img + gi * LH_IMG_AS + gj, v);
            } else if (prm.bimg) {
                // k_ctrl_b's band image (prm.bimg): the lower slot, (row, column) = (6q + bb, 6p + a) for p < q
                const int gi = 6 * p + a, gj = 6 * q + bb, r_ = (p < q) ? gj : gi, c_ = (p < q) ? gi : gj;
                if ((p < q || a >= bb) && lh_bimg_in(r_, c_)) st_red(img + lh_bimg_idx(r_, c_), v);
            } else {
                st_red(rs + LY.off_S + b * 36 + lane, v);
            }
            if (diag && a == bb) st_red(rs + LY.off_hd + 6 * p + a, h);
        }
        // b_p (lanes 36..41) and bs = b_p - bsd (needs lane + 6)
        const double bsd = __shfl_down(h, 6);
        if (diag && lane >= 36 && lane < 42) {
            st_red(rs + LY.off_bp + 6 * p + (lane - 36), h);
            st_red(rs + LY.off_bs + 6 * p + (lane - 36), h - bsd);
            if (prm.img) st_red(img + LH_NPAD * LH_IMG_AS + 6 * p + (lane - 36), h - bsd);   // the rhs row
        }
    }
    STAMP(20);
    STAMP_FLUSH(20, 1);
}

// ============================================================================
// k_ctrl: LM controller + reduced-system solve, one workgroup of 1024 threads (16 waves: the
// LDLT's trailing updates are latency-bound MFMA chains, four waves per SIMD overlap them).
//
//  1. one global round trip: every thread prefetches its slice of the staged reduced system and
//     the LM decision k_reduce took (one rank: prm.dec_in_reduce); otherwise thread 0 runs
//     isGoodStepInLM behind the prefetch (the initial linearisation, sharded solves);
//  2. the chosen system (the committed one on a rejection) is scattered straight from registers
//     into LDS in natural pose order, lambda on the diagonal (problem.cpp:408-418), committing it on
//     accept.  The solve is LDL^T without pivoting: S + lambda D is symmetric positive
//     (semi)definite, where Eigen's LDLT (problem.cpp:420) pivots on the largest diagonal; the two
//     agree to rounding (a zero pivot -- a fixed pose under STRATEGY1 -- is skipped as Eigen's
//     pivot_is_valid does, and its component solved as 0);
//  3. right-looking blocked LDL^T (8-column blocks, one barrier per block) over the envelope of S
//     only (lh_ctrl_units), see lds_ldlt_solve; the right-hand side rides along as row NP;
//  4. blocked back substitution in one wave; the step and the gain's pose part.
// The matrix is padded to NE = ceil16(n) with identity rows: no bounds tests in the inner loops.
// ============================================================================
#define CT 1024
#define NP LH_NPAD            // padded system size; row NP of A holds the right-hand side
#define AS (LH_NPAD + 2)      // LDS row stride, = 2 mod 32 doubles: a 16x4 tile fragment (lane (i, k) at row i,
                              // column k) hits 32 distinct 8-byte bank pairs per half-wave (ds_read_b64 banks
                              // (a/4) mod 64 over lanes 0-31 / 32-63); the odd stride 129 put rows i and i + 1 at
                              // columns k + 1 and k on one pair (two-way conflicts on every tile read)
#define RS_MAX (LH_PMAX * (LH_PMAX + 1) / 2 * 36 + 18 * LH_PMAX + 8)
#define ER 1008               // reduced-system elements per prefetch round: 28 whole 6x6 S blocks
#define NLD ((RS_MAX + ER - 1) / ER)
#define NBLK (LH_NPAD / 8)

// Per-block products of the 8x8 diagonal-block factor (LDS, shared by all waves).
struct LdltBlockLds {
    double N[4][64];          // N = (Delta L^T)^-1 of the block being eliminated (row-major), by step parity
                              // (the two-chain schedule: chain c uses N[2c + parity])
    double ND[NBLK][64];      // N Delta = L_bb^-T of every block (row-major): trailing-update operand
                              // and the back substitution's block solve
    double z[NP];             // z = D^-1 L^-1 b (zero where |D| <= DBL_MIN)
};
// one instance per kernel, whichever schedule runs
__device__ __forceinline__ LdltBlockLds& ldlt_lds() {
    __shared__ __attribute__((aligned(16))) LdltBlockLds F;
    return F;
}

// 64-bit broadcast of lane L of each 16-lane row: one v_mov_b64_dpp row_newbcast (gfx950 allows 64-bit DPP
// for row_newbcast).  The factor and the back substitution are issue-bound chains of these (a lone wave
// issues a dependent f64 op every ~7-10 cycles), so one move instead of two 32-bit halves is what counts.
template <int L>
__device__ __forceinline__ double bcast16(double v) {
    const long long x = __builtin_amdgcn_update_dpp((long long)0, __double_as_longlong(v), 0x150 + L, 0xf, 0xf, true);
    return __longlong_as_double(x);
}

// Column Q of the 8x8 factor: the pivot from lane Q by broadcast, its reciprocal (v_rcp_f64 and two
// Newton steps), the column's entries and the trailing updates of the lane's row.  (A cubic correction
// folded into the quotient, three dependent FMAs instead of five, measured the same ~1.8k cycles per
// block alone, tools/ubench_ctrl_chain.hip: the chain is bound by issue, not by this latency.)
// SAFE: Eigen ldlt_inplace's zero-pivot rule (no scaling where !pivot_is_valid: Delta = 1) on the chain;
// the fast form takes every pivot as valid and factor_block8_v redoes the block in the safe form when one
// was not (a fixed pose under STRATEGY1), so valid blocks get the same bits with three fewer dependent
// instructions per column.
template <int Q, bool SAFE>
__device__ __forceinline__ void factor_column(double (&R)[8], double (&dl)[8]) {
    const double d = bcast16<Q>(R[Q]);
    dl[Q] = SAFE ? (fabs(d) > 0.0 ? d : 1.0) : d;
    const double inv = fast_rcp(dl[Q]);
    const double coef = R[Q] * inv;
    double u[8];
    // W[j][Q] = lane j's R[Q], read before R[Q] becomes coef
    if (Q < 1) u[1] = bcast16<1>(R[Q]);
    if (Q < 2) u[2] = bcast16<2>(R[Q]);
    if (Q < 3) u[3] = bcast16<3>(R[Q]);
    if (Q < 4) u[4] = bcast16<4>(R[Q]);
    if (Q < 5) u[5] = bcast16<5>(R[Q]);
    if (Q < 6) u[6] = bcast16<6>(R[Q]);
    if (Q < 7) u[7] = bcast16<7>(R[Q]);
#pragma unroll
    for (int j = Q + 1; j < 8; ++j) R[j] -= coef * u[j];
    R[Q] = coef;
}

// Where the blocked LDL^T keeps its operands (the same code serves both controllers):
//  LdsSys  (k_ctrl, n <= LH_NPAD): the whole system in LDS, row stride AS, the rhs as row NP, L^T in
//          the upper triangle (L[r][c] at A[c][r]) for the back substitution;
//  BandSys (k_ctrl_b, banded windows past LH_PMAX poses): a 128-row circular window of the lower band
//          in LDS (row r at r mod 128, column c at c mod 128: no two live entries of a band narrower
//          than the window share a slot), the rhs in its own LDS array, L rows to global memory
//          (L[r][c] at Lg[r * LH_LBW + c - r + LH_LBW], c in [r - LH_LBW, r)).
struct LdsSys {
    // the trailing stores rewrite the entries outside the update with their own value (one exec mask
    // for the four stores; k_ctrl 28.09 / 28.04 -> 27.46 / 27.54 us); in k_ctrl_b's busier LDS (the
    // stream loaders' writes) the extra stores measured slower, so BandSys keeps the per-entry masks
    static constexpr bool rewrite_masked = true;
    double* A;
    __device__ __forceinline__ double& at(int r, int c) const { return A[r * AS + c]; }
    __device__ __forceinline__ double& rhs(int r) const { return A[NP * AS + r]; }
    __device__ __forceinline__ void store_l(int r, int c, double v) const { A[c * AS + r] = v; }
    // indices as stored: a 16-row tile row or 8-column block starts at a multiple of 8, so wrapping its
    // base once wraps every row / column of it (no carry into the base)
    __device__ __forceinline__ int wrap(int x) const { return x; }
    __device__ __forceinline__ double& atw(int r, int c) const { return A[r * AS + c]; }
};
#define LH_LBW 128   // k_ctrl_b: L entries kept per row (columns r - 128 .. r - 1)
struct BandSys {
    static constexpr bool rewrite_masked = false;
    double* A;   // LDS, 128 rows of stride AS
    double* y;   // LDS rhs
    double* Lg;  // global, LH_LBW per row
    __device__ __forceinline__ double& at(int r, int c) const { return A[(r & 127) * AS + (c & 127)]; }
    __device__ __forceinline__ double& rhs(int r) const { return y[r]; }
    __device__ __forceinline__ void store_l(int r, int c, double v) const { Lg[(size_t)r * LH_LBW + (c - r + LH_LBW)] = v; }
    __device__ __forceinline__ int wrap(int x) const { return x & 127; }
    __device__ __forceinline__ double& atw(int r, int c) const { return A[r * AS + c]; }
};

// LDL^T of the 8x8 diagonal block at (k0, k0) of A by one wave, Eigen ldlt_inplace order (L = W
// where pivot_is_valid fails).  In each 16-lane row (four identical replicas), lane r < 8 holds
// row r of the block and lane 8 + r row r of the identity: the same column eliminations turn
// the first into L and the second into N = (Delta L^T)^-1, Delta = diag(D, 1 where invalid), so
// one instruction stream computes both.  Column q's pivot and entries move by DPP broadcast.
// Writes D on A's diagonal and L^T above it (L[r][c] at A[c][r]), N, and ND = N Delta = L^-T.
// For a row a below the block, l = a N is its forward substitution through the block and
// l Delta its partially eliminated entries, so the trailing update of rows i, j is
// L_i Delta L_j^T = T_i a_j^T with T_i = L_i ND^T.
// v: row r = lane & 7 of the block (entries past the diagonal unused)
template <class S>
__device__ __forceinline__ void factor_block8_v(const S& A, const double (&v)[8], double* __restrict__ No,
                                                double* __restrict__ NDo, int k0, int lane) {
    const int p = lane & 15, r = p & 7;
    const bool ident = p >= 8;
    double R[8], dl[8];
    const int kw = A.wrap(k0);
#pragma unroll
    for (int q = 0; q < 8; ++q) R[q] = ident ? (q == r ? 1.0 : 0.0) : v[q];
    factor_column<0, false>(R, dl);
    factor_column<1, false>(R, dl);
    factor_column<2, false>(R, dl);
    factor_column<3, false>(R, dl);
    factor_column<4, false>(R, dl);
    factor_column<5, false>(R, dl);
    factor_column<6, false>(R, dl);
    factor_column<7, false>(R, dl);
    bool ok = true;   // every pivot valid (the pivots are the same in every lane)
#pragma unroll
    for (int q = 0; q < 8; ++q) ok = ok && fabs(dl[q]) > 0.0;
    if (!__builtin_amdgcn_readfirstlane(ok)) {   // rare: redo the block with the zero-pivot rule
#pragma unroll
        for (int q = 0; q < 8; ++q) R[q] = ident ? (q == r ? 1.0 : 0.0) : v[q];
        factor_column<0, true>(R, dl);
        factor_column<1, true>(R, dl);
        factor_column<2, true>(R, dl);
        factor_column<3, true>(R, dl);
        factor_column<4, true>(R, dl);
        factor_column<5, true>(R, dl);
        factor_column<6, true>(R, dl);
        factor_column<7, true>(R, dl);
    }
    if (lane < 8) {
        if constexpr (S::rewrite_masked) {
            // no branch per store: the entries below the diagonal go to the row's padding column
            // (LH_NPAD, never read)
#pragma unroll
            for (int q = 0; q < 8; ++q) A.atw(kw + q, q <= r ? kw + r : LH_NPAD) = (q == r) ? dl[q] : R[q];
        } else {
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (q <= r) A.atw(kw + q, kw + r) = (q == r) ? dl[q] : R[q];
        }
    } else if (lane < 16) {
        double2* n2 = reinterpret_cast<double2*>(No + 8 * r);
        double2* d2 = reinterpret_cast<double2*>(NDo + 8 * r);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            n2[q] = double2{R[2 * q], R[2 * q + 1]};
            d2[q] = double2{R[2 * q] * dl[2 * q], R[2 * q + 1] * dl[2 * q + 1]};
        }
    }
}
template <class S>
__device__ __forceinline__ void factor_block8(const S& A, double* __restrict__ No, double* __restrict__ NDo, int k0,
                                              int lane) {
    const int r = lane & 7, kw = A.wrap(k0);
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = A.atw(kw + r, kw + q);   // upper entries: garbage confined to this lane's upper part
    factor_block8_v(A, v, No, NDo, k0, lane);
}

// Step k0 of the elimination for the 16-row tile row at rb (one wave): with the raw block column
// a_I = A[rb..rb+15][k0..k0+7] (rows below k0+8 only; the block's own rows are masked),
//   L_I^T = N^T a_I^T              (MFMA; lands in A-operand layout: lane (li, lk) holds L[li][lk], L[li][lk+4])
//   T_I^T = ND L_I^T               (T_I = L_I Delta N^T, again in A-operand layout)
//   L^T -> A[k0+c][i]              (upper triangle; only when store_l)
//   b_i -= T_I . b_blk             (forward substitution of the rhs row; only when store_l)
//   A_IJ -= T_I a_J^T  for the tile columns J in [jb0, jb1) except skip_cb (lower part, cols >= m0).
// Every operand is the block column as it was before this step: no panel pass and no barrier
// between the elimination of the column and the trailing update.
template <class S>
__device__ __forceinline__ void ldlt_tile_row(const S& A, const double* __restrict__ N, const double* __restrict__ ND,
                                              int k0, int rb, int jb0, int jb1, int skip_cb, bool store_l, int lane) {
    const int li = lane & 15, lk = lane >> 4, m0 = k0 + 8;
    const int rbw = A.wrap(rb), kw = A.wrap(k0);
    const bool lo = li < 8;
    // every LDS read of this tile row is issued up front (tiles are disjoint and this step's
    // writes never touch block column k0, so no read here can see a write of this step)
    // (unconditional reads, selected after: no exec-masked branches between the loads)
    const double n0 = N[lk * 8 + (li & 7)], n1 = N[(lk + 4) * 8 + (li & 7)];
    const double d0 = ND[(li & 7) * 8 + lk], d1 = ND[(li & 7) * 8 + 4 + lk];
    const double a0 = A.atw(rbw + li, kw + lk), a1 = A.atw(rbw + li, kw + 4 + lk);
    const double na0 = lo ? n0 : 0.0, na1 = lo ? n1 : 0.0, da0 = lo ? d0 : 0.0, da1 = lo ? d1 : 0.0;
    int cb = (jb0 == skip_cb) ? jb0 + 16 : jb0;
    double b0 = 0.0, b1 = 0.0, old[4] = {0.0, 0.0, 0.0, 0.0};
    if (cb < jb1) {
        const int cbw = A.wrap(cb);
        b0 = A.atw(cbw + li, kw + lk);
        b1 = A.atw(cbw + li, kw + 4 + lk);
#pragma unroll
        for (int q = 0; q < 4; ++q) old[q] = A.atw(rbw + li, cbw + lk + 4 * q);
    }
    __builtin_amdgcn_sched_barrier(0);   // every load above is in flight before the first wait
    v4d l = {0.0, 0.0, 0.0, 0.0};
    l = __builtin_amdgcn_mfma_f64_16x16x4f64(na0, a0, l, 0, 0, 0);
    l = __builtin_amdgcn_mfma_f64_16x16x4f64(na1, a1, l, 0, 0, 0);
    // l[q] = L[rb+li][k0+lk+4q] (q = 0, 1)
    v4d t = {0.0, 0.0, 0.0, 0.0};
    t = __builtin_amdgcn_mfma_f64_16x16x4f64(da0, l[0], t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f64_16x16x4f64(da1, l[1], t, 0, 0, 0);
    // t[q] = T[rb+li][lk+4q] (q = 0, 1)
    if (store_l) {
        const double rb0 = (li == 0) ? A.rhs(k0 + lk) : 0.0, rb1 = (li == 0) ? A.rhs(k0 + 4 + lk) : 0.0;
        double rold[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) rold[q] = A.rhs(rb + lk + 4 * q);
        if (rb + li >= m0) {
            A.store_l(rb + li, k0 + lk, l[0]);
            A.store_l(rb + li, k0 + 4 + lk, l[1]);
        }
        v4d u = {0.0, 0.0, 0.0, 0.0};
        u = __builtin_amdgcn_mfma_f64_16x16x4f64(t[0], rb0, u, 0, 0, 0);
        u = __builtin_amdgcn_mfma_f64_16x16x4f64(t[1], rb1, u, 0, 0, 0);
        // u[q] = (T b_blk)[rb+lk+4q] in column li = 0
        if (li == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = rb + lk + 4 * q;
                if (row >= m0) A.rhs(row) = rold[q] - u[q];
            }
        }
    }
    // trailing tiles, software-pipelined: the next tile's operands are in flight during this one's MFMAs
    while (cb < jb1) {
        const int cbw_cur = A.wrap(cb);
        int nc = cb + 16;
        if (nc == skip_cb) nc += 16;
        double nb0 = 0.0, nb1 = 0.0, nold[4] = {0.0, 0.0, 0.0, 0.0};
        if (nc < jb1) {
            const int ncw = A.wrap(nc);
            nb0 = A.atw(ncw + li, kw + lk);
            nb1 = A.atw(ncw + li, kw + 4 + lk);
#pragma unroll
            for (int q = 0; q < 4; ++q) nold[q] = A.atw(rbw + li, ncw + lk + 4 * q);
        }
        // the update transposed, (a_J T_I^T)^T: lane (li, lk) gets row li, columns lk + 4q of the tile, the
        // same fragment shape as the operand reads (conflict-free at this stride); the products are the
        // same, so are the bits
        v4d acc = {0.0, 0.0, 0.0, 0.0};
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(b0, t[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(b1, t[1], acc, 0, 0, 0);
        const int row = rb + li;
        // entries outside the update (left of m0, above the diagonal) get their own value back: no other
        // wave writes them this step, and the four stores share one exec mask instead of four branches
        if constexpr (S::rewrite_masked) {
            if (row >= m0) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int col = cb + lk + 4 * q;
                    A.atw(rbw + li, cbw_cur + lk + 4 * q) = (col >= m0 && col <= row) ? old[q] - acc[q] : old[q];
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int col = cb + lk + 4 * q;
                if (row >= m0 && col >= m0 && col <= row) A.atw(rbw + li, cbw_cur + lk + 4 * q) = old[q] - acc[q];
            }
        }
        cb = nc;
        b0 = nb0; b1 = nb1;
#pragma unroll
        for (int q = 0; q < 4; ++q) old[q] = nold[q];
    }
}

// Wave 0's share of step k0: the trailing update of the diagonal tile at rb (the one holding block
// k0 + 8), the head of every step's critical chain (this, then the next block's factor).  The
// operands are ldlt_tile_row's with a_J = a_I (the tile is its own column), so the eight LDS reads go
// out in one batch, unconditionally (N / ND rows past 7 read the neighbouring in-bounds LDS and are
// dropped by the select), and the only waits are the one round trip and the MFMA chain.
template <class S>
__device__ __forceinline__ void diag_tile(const S& A, const double* __restrict__ N, const double* __restrict__ ND,
                                          int k0, int rb, int lane) {
    const int li = lane & 15, lk = lane >> 4, m0 = k0 + 8;
    const int rbw = A.wrap(rb), kw = A.wrap(k0);
    const bool lo = li < 8;
    const double n0 = N[lk * 8 + (li & 7)], n1 = N[(lk + 4) * 8 + (li & 7)];
    const double d0 = ND[(li & 7) * 8 + lk], d1 = ND[(li & 7) * 8 + 4 + lk];
    const double a0 = A.atw(rbw + li, kw + lk), a1 = A.atw(rbw + li, kw + 4 + lk);
    double old[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) old[q] = A.atw(rbw + li, rbw + lk + 4 * q);
    __builtin_amdgcn_sched_barrier(0);   // the scheduler otherwise sinks the loads between the MFMAs
    v4d l = {0.0, 0.0, 0.0, 0.0};
    l = __builtin_amdgcn_mfma_f64_16x16x4f64(lo ? n0 : 0.0, a0, l, 0, 0, 0);
    l = __builtin_amdgcn_mfma_f64_16x16x4f64(lo ? n1 : 0.0, a1, l, 0, 0, 0);
    v4d t = {0.0, 0.0, 0.0, 0.0};
    t = __builtin_amdgcn_mfma_f64_16x16x4f64(lo ? d0 : 0.0, l[0], t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f64_16x16x4f64(lo ? d1 : 0.0, l[1], t, 0, 0, 0);
    v4d acc = {0.0, 0.0, 0.0, 0.0};   // transposed, as in ldlt_tile_row
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, t[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, t[1], acc, 0, 0, 0);
    const int row = rb + li;
    // as ldlt_tile_row: the entries outside the update are rewritten with their own value (above the
    // diagonal this wave's factor writes L^T next; rows above m0 are the store unit's, left alone)
    if constexpr (S::rewrite_masked) {
        if (row >= m0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int col = rb + lk + 4 * q;
                A.atw(rbw + li, rbw + lk + 4 * q) = (col >= m0 && col <= row) ? old[q] - acc[q] : old[q];
            }
        }
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int col = rb + lk + 4 * q;
            if (row >= m0 && col >= m0 && col <= row) A.atw(rbw + li, rbw + lk + 4 * q) = old[q] - acc[q];
        }
    }
}

// k_ctrl's two-chain steps (lh_ctrl_nd_plan): one tile row's unit applying up to two sources, the blocks
// the two chains eliminate this step.  For each source s in smask | stmask: L_s = a_s N_s, T_s = L_s ND_s^T
// with the rows above its block (< m0_s) zeroed, so they contribute nothing; stmask: L_s^T stored for the
// tile row and the rhs row updated by every stored source at once (two units never update one rhs row
// in a step); then A_IJ -= sum_{s in smask} T_s a_{s,J}^T over the tiles [jb0, jb1), a_{s,J}'s rows above
// the block zeroed likewise.  Entries above every applied source's block are left alone.
struct NdSrc {
    const double* N;
    const double* ND;
    int k0;
};
__device__ __forceinline__ void nd_tile_row(double* __restrict__ A, const NdSrc (&src)[2], int smask, int stmask, int rb,
                                            int jb0, int jb1, int lane) {
    const int li = lane & 15, lk = lane >> 4;
    const bool lo = li < 8;
    double t0[2], t1[2];
    int mm = 1 << 20;
    double ru[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        t0[q] = 0.0; t1[q] = 0.0;
        if (!(((smask | stmask) >> q) & 1)) continue;   // a stored source need not reach the unit's tiles
        const int k0 = src[q].k0, m0 = k0 + 8;
        mm = min(mm, m0);
        const double* N = src[q].N;
        const double* ND = src[q].ND;
        const double na0 = lo ? N[lk * 8 + li] : 0.0, na1 = lo ? N[(lk + 4) * 8 + li] : 0.0;
        const double da0 = lo ? ND[li * 8 + lk] : 0.0, da1 = lo ? ND[li * 8 + 4 + lk] : 0.0;
        const double a0 = A[(rb + li) * AS + k0 + lk], a1 = A[(rb + li) * AS + k0 + 4 + lk];
        v4d l = {0.0, 0.0, 0.0, 0.0};
        l = __builtin_amdgcn_mfma_f64_16x16x4f64(na0, a0, l, 0, 0, 0);
        l = __builtin_amdgcn_mfma_f64_16x16x4f64(na1, a1, l, 0, 0, 0);
        v4d t = {0.0, 0.0, 0.0, 0.0};
        t = __builtin_amdgcn_mfma_f64_16x16x4f64(da0, l[0], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f64_16x16x4f64(da1, l[1], t, 0, 0, 0);
        const bool below = rb + li >= m0;
        t0[q] = below ? t[0] : 0.0;
        t1[q] = below ? t[1] : 0.0;
        if ((stmask >> q) & 1) {
            if (below) {
                A[(k0 + lk) * AS + rb + li] = l[0];
                A[(k0 + 4 + lk) * AS + rb + li] = l[1];
            }
            const double rb0 = (li == 0) ? A[NP * AS + k0 + lk] : 0.0, rb1 = (li == 0) ? A[NP * AS + k0 + 4 + lk] : 0.0;
            v4d u = {0.0, 0.0, 0.0, 0.0};
            u = __builtin_amdgcn_mfma_f64_16x16x4f64(t0[q], rb0, u, 0, 0, 0);
            u = __builtin_amdgcn_mfma_f64_16x16x4f64(t1[q], rb1, u, 0, 0, 0);
#pragma unroll
            for (int w = 0; w < 4; ++w) ru[w] += u[w];
        }
    }
    if (stmask && li == 0) {
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int row = rb + lk + 4 * w;
            if (row >= mm) A[NP * AS + row] -= ru[w];
        }
    }
    for (int cb = jb0; cb < jb1; cb += 16) {
        double old[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) old[w] = A[(rb + li) * AS + cb + lk + 4 * w];
        v4d acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            if (!((smask >> q) & 1)) continue;
            const int k0 = src[q].k0, m0 = k0 + 8;
            const bool cin = cb + li >= m0;
            const double b0 = cin ? A[(cb + li) * AS + k0 + lk] : 0.0, b1 = cin ? A[(cb + li) * AS + k0 + 4 + lk] : 0.0;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(b0, t0[q], acc, 0, 0, 0);   // transposed
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(b1, t1[q], acc, 0, 0, 0);
        }
        const int row = rb + li;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int col = cb + lk + 4 * w;
            if (row >= mm && col >= mm && col <= row) A[row * AS + col] = old[w] - acc[w];
        }
    }
}

// Back substitution x = L^-T z for block KB (compile-time, so every lane index below is an
// immediate), one wave: y holds rows lane (y0) and lane + 64 (y1), already reduced by every block
// above KB.  x_b = ND_b y_b: the block's 8 y values sit in lanes KB..KB+7 (mod 64), inside one
// 16-lane row, and reach that row's lanes by DPP broadcast; lane KB+v computes x_b[v], so it
// holds its own row's result.  Every row r above the block then takes y_r -= sum_v L[KB+v][r]
// x_b[v] (L^T row r in the upper triangle), x_b broadcast by readlane.  No LDS writes: the
// compiler may hoist every block's operand loads.
// The LDS operands of the back substitution never change while it runs, so no load waits for the
// chain: the caller loads block b-1's ND_b row while block b computes, and each block issues its L^T
// loads before its first DPP broadcast (all unconditional: a block past nb reads in-bounds padding it
// never uses).  Loading them after the runtime nb guard put two dependent LDS round trips on the
// chain per block: the compiler does not hoist loads across those branches.
template <int KB>
__device__ __forceinline__ void backsub_load_nd(const LdltBlockLds& F, int lane, double (&nd)[8]) {
#pragma unroll
    for (int w = 0; w < 8; ++w) nd[w] = F.ND[KB >> 3][(lane & 7) * 8 + w];
}

// Back substitution x = L^-T z for block KB (compile-time, so every lane index below is an
// immediate), one wave: y holds rows lane (y0) and lane + 64 (y1), already reduced by every block
// above KB.  x_b = ND_b y_b: the block's 8 y values sit in lanes KB..KB+7 (mod 64), inside one
// 16-lane row, and reach that row's lanes by DPP broadcast; lane KB+v computes x_b[v], so it
// holds its own row's result.  Every row r above the block then takes y_r -= sum_v L[KB+v][r]
// x_b[v] (L^T row r in the upper triangle), x_b broadcast by readlane.
template <int KB>
__device__ __forceinline__ void backsub_block(const double* __restrict__ A, const double (&nd)[8], int nb, int lane,
                                              double& y0, double& y1) {
    constexpr bool HI = KB >= 64;
    constexpr int KL = KB & 63, R16 = KL & 15;
    double l0[8], l1[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) l0[v] = A[lane * AS + KB + v];
    if (HI) {
#pragma unroll
        for (int v = 0; v < 8; ++v) l1[v] = A[(lane + 64) * AS + KB + v];
    }
    // the loads stay ahead of the broadcasts (left alone, the scheduler sinks them past the nb branch to
    // their first use, after x_b, and the LDS round trip lands on the chain)
    __builtin_amdgcn_sched_barrier(0);
    if (KB >= nb) return;
    const double ys = HI ? y1 : y0;
    double yb[8];
    yb[0] = bcast16<R16 + 0>(ys); yb[1] = bcast16<R16 + 1>(ys); yb[2] = bcast16<R16 + 2>(ys); yb[3] = bcast16<R16 + 3>(ys);
    yb[4] = bcast16<R16 + 4>(ys); yb[5] = bcast16<R16 + 5>(ys); yb[6] = bcast16<R16 + 6>(ys); yb[7] = bcast16<R16 + 7>(ys);
    const double xv = ((nd[0] * yb[0] + nd[1] * yb[1]) + (nd[2] * yb[2] + nd[3] * yb[3])) +
                      ((nd[4] * yb[4] + nd[5] * yb[5]) + (nd[6] * yb[6] + nd[7] * yb[7]));
    double xb[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) xb[v] = readlane_d(xv, KL + v);
    const double s0 = ((l0[0] * xb[0] + l0[1] * xb[1]) + (l0[2] * xb[2] + l0[3] * xb[3])) +
                      ((l0[4] * xb[4] + l0[5] * xb[5]) + (l0[6] * xb[6] + l0[7] * xb[7]));
    if (HI) {
        const double s1 = ((l1[0] * xb[0] + l1[1] * xb[1]) + (l1[2] * xb[2] + l1[3] * xb[3])) +
                          ((l1[4] * xb[4] + l1[5] * xb[5]) + (l1[6] * xb[6] + l1[7] * xb[7]));
        y0 -= s0;
        y1 = (lane + 64 < KB) ? y1 - s1 : ((lane + 64 < KB + 8) ? xv : y1);
    } else {
        y0 = (lane < KB) ? y0 - s0 : ((lane < KB + 8) ? xv : y0);
    }
}

// Phase 4 of both LDL^T schedules: x = L^-T z over every block, descending, one wave (y0 / y1: rows
// lane / lane + 64 of z in, of x out, in the factor's order).
__device__ __forceinline__ void ldlt_backsub(const double* __restrict__ A, const LdltBlockLds& F, int nb, int lane,
                                             double& y0, double& y1) {
    double nda[8], ndb[8];
    backsub_load_nd<120>(F, lane, nda);
    backsub_load_nd<112>(F, lane, ndb);
    backsub_block<120>(A, nda, nb, lane, y0, y1);
    backsub_load_nd<104>(F, lane, nda);
    backsub_block<112>(A, ndb, nb, lane, y0, y1);
    backsub_load_nd<96>(F, lane, ndb);
    backsub_block<104>(A, nda, nb, lane, y0, y1);
    backsub_load_nd<88>(F, lane, nda);
    backsub_block<96>(A, ndb, nb, lane, y0, y1);
    backsub_load_nd<80>(F, lane, ndb);
    backsub_block<88>(A, nda, nb, lane, y0, y1);
    backsub_load_nd<72>(F, lane, nda);
    backsub_block<80>(A, ndb, nb, lane, y0, y1);
    backsub_load_nd<64>(F, lane, ndb);
    backsub_block<72>(A, nda, nb, lane, y0, y1);
    backsub_load_nd<56>(F, lane, nda);
    backsub_block<64>(A, ndb, nb, lane, y0, y1);
    backsub_load_nd<48>(F, lane, ndb);
    backsub_block<56>(A, nda, nb, lane, y0, y1);
    backsub_load_nd<40>(F, lane, nda);
    backsub_block<48>(A, ndb, nb, lane, y0, y1);
    backsub_load_nd<32>(F, lane, ndb);
    backsub_block<40>(A, nda, nb, lane, y0, y1);
    backsub_load_nd<24>(F, lane, nda);
    backsub_block<32>(A, ndb, nb, lane, y0, y1);
    backsub_load_nd<16>(F, lane, ndb);
    backsub_block<24>(A, nda, nb, lane, y0, y1);
    backsub_load_nd<8>(F, lane, nda);
    backsub_block<16>(A, ndb, nb, lane, y0, y1);
    backsub_load_nd<0>(F, lane, ndb);
    backsub_block<8>(A, nda, nb, lane, y0, y1);
    backsub_block<0>(A, ndb, nb, lane, y0, y1);
}

// The controller's step tail taken by the back-substitution wave from its registers (k_ctrl, LDL^T): the
// pose part of the gain denominator (isGoodStepInLM's scale, problem.cpp:528-533) summed over the wave
// (rows lane and lane + 64 of one lane first), the step stored for k_lin.  ctrl null: no tail (the probe).
struct LdltTail {
    lh_ctrl* ctrl;
    double* dxp;
    const double* bpv;
    const double* hdv;
    double lambda;
    int strategy;
    int rung;   // the lambda-ladder rung this controller workgroup solves (lh_ctrl.spose_l)
};
__device__ __forceinline__ void ldlt_tail(const LdltTail& tl, int n, int lane, double y0, double y1) {
    auto term = [&](int r, double d) {
        if (r >= n) return 0.0;
        if (tl.dxp) tl.dxp[r] = d;
        const double b = tl.bpv[r];
        return (tl.strategy == 0) ? d * (tl.lambda * d + b) : d * (tl.lambda * tl.hdv[r] * d + b);
    };
    double sp[1] = {term(lane, y0) + term(lane + 64, y1)};
    group_sum(sp, 6);
    if (lane == 0) tl.ctrl->spose_l[tl.rung] = sp[0];
}

// Phases 3-4 of k_ctrl on a padded system already in LDS (A lower + rhs row NP, zeros in the upper
// triangle): blocked LDL^T with the forward substitution, then the back substitution; xsol[perm[r]] =
// the solution's entry r < n (perm == nullptr: xsol[r]).  units: the per-step work units in LDS
// (lh_ctrl_units: the envelope of S decides which tile rows a step touches).  Shared with the
// k_ldlt_probe test hook.  Must be called by all CT threads.
//
// Step t eliminates block column k0 = 8t.  Interval t (one barrier each):
//   wave 0:       the trailing update of the diagonal tile holding block t+1 (when its envelope
//                 reaches block t), then the factor of block t+1 (N by step parity, ND per block);
//   waves 1-15:   their unit of step t: L_I (stored transposed), T_I, the rhs update and
//                 A_IJ -= T_I a_J^T over the unit's tile columns;
//   wave 12 first: z_t = b_t N_t (Eigen's solve tolerance applied).
// L lives in the upper triangle, so the raw block columns stay readable for the whole step.
__device__ __forceinline__ void lds_ldlt_solve(double* __restrict__ A, double* __restrict__ xsol, int n, int NE, int tid,
                                               const int* __restrict__ perm, const uint16_t* __restrict__ units,
                                               const LdltTail& tl = LdltTail{}, bool factored0 = false) {
    const int lane = tid & 63, wave = tid >> 6;
    LdltBlockLds& F = ldlt_lds();
    const int nb = (n + 7) & ~7;          // blocks past the last real row are identity: never eliminated
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const LdsSys SY{A};
    // this wave's unit words, lane t holding step t's: read once, so no step starts with an LDS round trip
    const uint32_t uwv = (lane < LH_NSTEP) ? units[wv * LH_NSTEP + lane] : 0u;
    if (!factored0) {   // (k_ctrl factors block 0 during its scatter)
        if (wv == 0) factor_block8(SY, F.N[0], F.ND[0], 0, lane);
        lds_barrier();
    }
    CSTAMP(5);
#ifdef LH_STAMPS
    // per-step split (diagnostic): wave 0's diagonal tile, its factor and its wait at the barrier;
    // the other waves' unit time and barrier wait (wave-cycles summed over waves)
    unsigned long long ss_[5] = {0, 0, 0, 0, 0}, sa_ = __builtin_amdgcn_s_memtime(), sb_;
    // per step t: [64 + t] wave 0's diagonal tile, [80 + t] its factor, [96 + t] its barrier wait
    // (sums over launches), [112 + t] the slowest other wave's unit in the worst launch (atomicMax of
    // cycles << 24 | unit word << 4 | wave)
    uint32_t su_ = 0;
#define LDLT_SSTAMP(i) do { __builtin_amdgcn_sched_barrier(0); sb_ = __builtin_amdgcn_s_memtime(); \
        ss_[i] += sb_ - sa_; \
        if (lane == 0 && (i) != 4) { \
            const int ti_ = min(k0 >> 3, 15); \
            if ((i) == 3) atomicMax(&lh_stamps[112 + ti_], ((sb_ - sa_) << 24) | ((unsigned long long)(su_ & 0xffffu) << 4) | (unsigned)wv); \
            else atomicAdd(&lh_stamps[64 + 16 * ((i) == 0 ? 0 : (i) == 1 ? 1 : 2) + ti_], sb_ - sa_); } \
        sa_ = sb_; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define LDLT_SSTAMP(i)
#endif
    for (int k0 = 0; k0 < nb; k0 += 8) {
        const int t = k0 >> 3, par = t & 1, m0 = k0 + 8;
        const double* N = F.N[par];
        const double* ND = F.ND[t];
        if (wv == 12 && lane < 8) {       // z_t = b_t N_t, zeroed where |D| <= DBL_MIN (LDLT::_solve_impl)
            double z = 0.0;
#pragma unroll
            for (int q = 0; q < 8; ++q) z += A[NP * AS + k0 + q] * N[q * 8 + lane];
            const double d = A[(k0 + lane) * AS + k0 + lane];
            F.z[k0 + lane] = fabs(d) > 2.2250738585072014e-308 ? z : 0.0;
        }
        if (m0 < nb) {
            const int g0 = m0 >> 4;               // tile row/col of the next diagonal block
            const uint32_t uw = __builtin_amdgcn_readlane(uwv, t);
#ifdef LH_STAMPS
            su_ = uw;
#endif
            if (wv == 0) {
                if (uw & LH_UNIT_VALID) {
                    diag_tile(SY, N, ND, k0, 16 * g0, lane);
                    wave_sync();
                }
                LDLT_SSTAMP(0);
                factor_block8(SY, F.N[par ^ 1], F.ND[t + 1], m0, lane);
                LDLT_SSTAMP(1);
            } else if (uw & LH_UNIT_VALID) {
                const int I = g0 + (uw & 7), jb0 = g0 + ((uw >> 3) & 7), jb1 = g0 + ((uw >> 6) & 15);
                ldlt_tile_row(SY, N, ND, k0, 16 * I, 16 * jb0, 16 * jb1, -1, (uw & LH_UNIT_STORE) != 0, lane);
            }
            if (wv != 0) LDLT_SSTAMP(3);
        }
        lds_barrier();
        if (wv == 0) LDLT_SSTAMP(2); else LDLT_SSTAMP(4);
    }
#ifdef LH_STAMPS
    if (lane == 0) {
        if (wv == 0) {
            atomicAdd(&lh_stamps[46], ss_[0]);
            atomicAdd(&lh_stamps[47], ss_[1]);
            atomicAdd(&lh_stamps[48], ss_[2]);
            atomicAdd(&lh_stamps[51], 1ull);
        } else {
            atomicAdd(&lh_stamps[49], ss_[3]);
            atomicAdd(&lh_stamps[50], ss_[4]);
        }
    }
#endif
    CSTAMP(6);

    // ---------------- 4. back substitution x = L^-T z, blocks descending, one wave ----------------
    if (wv == 0) {
        double y0 = (lane < nb) ? F.z[lane] : 0.0, y1 = (lane + 64 < nb) ? F.z[lane + 64] : 0.0;
        ldlt_backsub(A, F, nb, lane, y0, y1);
        if (perm) {
            if (lane < n) xsol[perm[lane]] = y0;
            if (lane + 64 < n) xsol[perm[lane + 64]] = y1;
        } else {
            if (lane < NE) xsol[lane] = y0;
            if (lane + 64 < NE) xsol[lane + 64] = y1;
        }
        if (tl.ctrl) ldlt_tail(tl, n, lane, y0, y1);
    }
    lds_barrier();
    CSTAMP(7);
}

// Phases 3-4 of k_ctrl, two-chain schedule (lh_ctrl_nd_plan): the system is in LDS in
// the order [long part | short part | separator] (lh_nd_pos), the two parts decoupled, so their LDL^T
// are independent chains.  Step t eliminates chain 0's block c0(t) (the long part's blocks, then the
// separator's) and chain 1's block c1(t) (the short part's, while they last); one barrier per step.
//   wave 0 / wave 1: the next diagonal tile of chain 0 / 1 (every source of the step reaching it), then
//                    that chain's next factor (N by chain and step parity, ND per block);
//   other waves:     their unit (nd_tile_row: up to both sources per tile, tile rows and columns absolute);
//   wave 12 / 13:    z of chain 0's / 1's block first.
// The back substitution is the one-chain one over the factor order; x goes out in natural order.
__device__ __forceinline__ void lds_ldlt_solve_nd(double* __restrict__ A, double* __restrict__ xsol, int n, int tid,
                                                  const uint16_t* __restrict__ units, const lh_params& prm) {
    const int lane = tid & 63, wave = tid >> 6;
    LdltBlockLds& F = ldlt_lds();
    const int nb = (n + 7) & ~7;
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const int P = prm.P, a = prm.nd_a, sep = prm.nd_s, lf = prm.nd_long_first, T = prm.nd_steps;
    const int b = P - a - sep;
    const int nl_blk = 6 * (lf ? a : b) / 8, ns_blk = 6 * (lf ? b : a) / 8;
    auto c0 = [&](int t) { return t < nl_blk ? t : t + ns_blk; };          // chain 0's block at step t
    auto c1 = [&](int t) { return t < ns_blk ? nl_blk + t : -1; };        // chain 1's (-1: done)
    const LdsSys SY{A};
    const uint32_t uwv = (lane < LH_NSTEP) ? units[wv * LH_NSTEP + lane] : 0u;   // lane t: step t's unit word
    if (wv == 0) factor_block8(SY, F.N[0], F.ND[c0(0)], 8 * c0(0), lane);
    if (wv == 1 && ns_blk > 0) factor_block8(SY, F.N[2], F.ND[c1(0)], 8 * c1(0), lane);
    lds_barrier();
    CSTAMP(5);
    for (int t = 0; t < T; ++t) {
        const int par = t & 1, ka = c0(t), kb = c1(t);
        const NdSrc src[2] = {{F.N[par], F.ND[ka], 8 * ka}, {F.N[2 + par], F.ND[kb < 0 ? 0 : kb], 8 * kb}};
        if ((wv == 12 || (wv == 13 && kb >= 0)) && lane < 8) {   // z of the step's blocks (LDLT::_solve_impl)
            const int q0 = wv == 12 ? 0 : 1, k0 = src[q0].k0;
            const double* N = src[q0].N;
            double z = 0.0;
#pragma unroll
            for (int q = 0; q < 8; ++q) z += A[NP * AS + k0 + q] * N[q * 8 + lane];
            const double d = A[(k0 + lane) * AS + k0 + lane];
            F.z[k0 + lane] = fabs(d) > 2.2250738585072014e-308 ? z : 0.0;
        }
        const uint32_t uw = __builtin_amdgcn_readlane(uwv, t);
        const int smask = (uw >> 10) & 3, stmask = (uw >> 12) & 3;
        if (wv < 2) {
            const int nx = wv == 0 ? c0(t + 1) : c1(t + 1);
            const bool live = wv == 0 ? (t + 1 < T) : (kb >= 0 && nx >= 0);
            if (uw & LH_UNIT_VALID) {
                const int I = uw & 7;
                nd_tile_row(A, src, smask, 0, 16 * I, 16 * I, 16 * I + 16, lane);
                wave_sync();
            }
            if (live) factor_block8(SY, F.N[2 * wv + (par ^ 1)], F.ND[nx], 8 * nx, lane);
        } else if (uw & LH_UNIT_VALID) {
            const int I = uw & 7, jb0 = (uw >> 3) & 7, jb1 = (uw >> 6) & 15;
            nd_tile_row(A, src, smask, stmask, 16 * I, 16 * jb0, 16 * jb1, lane);
        }
        lds_barrier();
    }
    CSTAMP(6);
    if (wv == 0) {
        double y0 = (lane < nb) ? F.z[lane] : 0.0, y1 = (lane + 64 < nb) ? F.z[lane + 64] : 0.0;
        ldlt_backsub(A, F, nb, lane, y0, y1);
        // factor row r -> natural row 6 nat(r / 6) + r mod 6
        if (lane < n) xsol[6 * lh_nd_nat(lane / 6, P, a, sep, lf) + lane % 6] = y0;
        if (lane + 64 < n) xsol[6 * lh_nd_nat((lane + 64) / 6, P, a, sep, lf) + (lane + 64) % 6] = y1;
    }
    lds_barrier();
    CSTAMP(7);
}

// Phases 3-4 of k_ctrl, PCG variant (lh_options.linear_solver = LH_SOLVER_PCG): Jacobi-preconditioned
// conjugate gradients on the same permuted, padded system (A lower triangle + rhs row NP).  This is
// the solver the reference left commented out (problem.cpp:421-422 -> Problem::PCGSolver :584-614)
// with its stop rule, ||r|| <= 1e-6 ||b|| (:597), and iteration cap, 2 * rows (:422), but corrected:
// the reference never adds the first step alpha*p to x (:595-596); here every step is applied.
// A zero diagonal entry (STRATEGY1 with a fixed pose: 0 + lambda*0) preconditions with 0 instead of
// Eigen's inf (which would turn the whole step into NaN).
// Layout: eight waves, the system cached in registers.  Wave w < 8 owns rows 16w .. 16w + 15; lane l
// holds row 16w + (l & 15) at columns 32 (l >> 4) + j, j < 32 (32 doubles).  A matrix-vector product is
// then 32 FMAs per lane on 16-byte broadcast reads of the vector, and a 2-level butterfly (lane ^ 16, 32) over
// the four lanes sharing a row; each row's scalars (x, r, z, p, q, 1/d) are replicated over those
// lanes.  Two workgroup barriers per step, the CG recurrence regrouped so that one product serves a
// step: with z published, q = A p = A z + beta q_prev and p = z + beta p_prev (the same iteration,
// rounded differently: parity to tolerance, as before).  The dot products are fixed-order sums
// (16-row wave butterflies, then the 8 wave partials in order), so a solve is bitwise repeatable.
// Waves 8-15 only keep the barrier count and the stop test (the r.r total, the same bits).  Per step
// the SIMD issue is what costs: all 16 waves doing the row scalars' replicated work took 1.85 us per
// step on C3; the round-2 layout (one wave, the system in LDS, an n-long FMA chain per row) ~2.5 us;
// round 1 (eight threads per row, three barriers) ~3 us.
// At most max_it steps (callers pass the reference cap + 1: its first step precedes its loop).
// Returns the iteration count.  Must be called by all CT threads; xsol[r] = x in pivot order.
__device__ __forceinline__ int lds_pcg_solve(double* __restrict__ A, double* __restrict__ xsol, double* __restrict__ pv,
                                             double* __restrict__ s_red2, int n, int tid, double tol_rel, int max_it) {
    constexpr int PW = 8;   // PCG waves
    static_assert(CT / 64 >= PW && NP == 16 * PW, "8 waves x 16 rows, 4 column blocks x 32");
    const int lane = tid & 63, wave = tid >> 6;
    const bool act = wave < PW;
    const int row = 16 * wave + (lane & 15), k = lane >> 4;
    const bool vr = act && row < n;
    double a[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const int c = 32 * k + j;
        a[j] = (vr && c < n) ? A[max(row, c) * AS + min(row, c)] : 0.0;   // S(i, j) = A[max * AS + min]
    }
    const double d = vr ? A[row * AS + row] : 0.0;
    const double id = (d != 0.0) ? 1.0 / d : 0.0;
    double r = vr ? A[NP * AS + row] : 0.0;
    double x = 0.0, z = r * id, p = 0.0, q = 0.0, beta = 0.0;
    double* red_pq = s_red2;                                            // [PW] wave partials of p.q
    double2* red_zr = reinterpret_cast<double2*>(s_red2 + 16);          // [PW] of (r.z, r.r)
    auto rows16 = [&](double v) {       // the wave's 16 rows (every lane gets the sum)
        double t[1] = {v};
        group_sum(t, 4);
        return t[0];
    };
    auto total = [&](const double* red) {   // in wave order
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < PW; ++w) t += red[w];
        return t;
    };
    auto total2 = [&](double& tz, double& tr) {
        tz = 0.0;
        tr = 0.0;
#pragma unroll
        for (int w = 0; w < PW; ++w) {
            const double2 t = red_zr[w];
            tz += t.x;
            tr += t.y;
        }
    };
    if (act) {
        if (k == 0 && row < NP) pv[row] = z;
        const double wrz = rows16(r * z), wrr = rows16(r * r);
        if (lane == 0) red_zr[wave] = double2{wrz, wrr};
    }
    lds_barrier();
    double rz, rr0;
    total2(rz, rr0);
    const double bnorm = sqrt(rr0);
    const double thr = tol_rel * bnorm;
    int it = 0;
    if (bnorm > 0.0) {
#pragma clang loop unroll(disable)
        while (it < max_it) {
            if (act) {
                // s = A z (z published in pv), then q = s + beta q, p = z + beta p
                double sp[4] = {0.0, 0.0, 0.0, 0.0};
                const double2* pz = reinterpret_cast<const double2*>(pv + 32 * k);
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const double2 v = pz[j];
                    sp[(2 * j) & 3] += a[2 * j] * v.x;
                    sp[(2 * j + 1) & 3] += a[2 * j + 1] * v.y;
                }
                double sv = (sp[0] + sp[1]) + (sp[2] + sp[3]);
                sv = xor16_sum(sv);
                sv = xor32_sum(sv);
                q = sv + beta * q;
                p = z + beta * p;
                const double wpq = rows16(vr ? p * q : 0.0);
                if (lane == 0) red_pq[wave] = wpq;
            }
            lds_barrier();
            if (act) {
                const double alpha = rz / total(red_pq);
                x += alpha * p;
                r -= alpha * q;
                z = r * id;
                const double wrz = rows16(vr ? r * z : 0.0), wrr = rows16(vr ? r * r : 0.0);
                if (lane == 0) red_zr[wave] = double2{wrz, wrr};
                if (k == 0 && row < NP) pv[row] = z;
            }
            lds_barrier();
            ++it;
            double rzn, rrn;
            total2(rzn, rrn);
            if (!(sqrt(rrn) > thr)) break;   // also stops on NaN; the same bits in every wave
            beta = rzn / rz;
            rz = rzn;
        }
    }
    if (k == 0 && vr) xsol[row] = x;
    lds_barrier();
    return it;
}

// The controllers' tail (xs: the pose step in pose order, in LDS): the pose part of the gain
// denominator (isGoodStepInLM's scale, problem.cpp:528-533), the wave partials summed in wave order
// into ctrl->spose_l[rung], and (dxp non-null) the step stored for k_lin.  The candidate poses
// (VertexPose::add) are built by the next k_lin (d_pose_candidate).  All NT threads.
template <int NT>
__device__ __forceinline__ void ctrl_step_tail(lh_ctrl* __restrict__ ctrl, const lh_params& prm, int n, double lambda,
                                               const double* xs, const double* bpv, const double* hdv, double* s_red,
                                               double* __restrict__ dxp, int rung = 0) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double sp = 0.0;
    for (int i = tid; i < n; i += NT) {
        const double d = xs[i], b = bpv[i];
        sp += (prm.strategy == 0) ? d * (lambda * d + b) : d * (lambda * hdv[i] * d + b);
        if (dxp) dxp[i] = d;
    }
    for (int off = 32; off > 0; off >>= 1) sp += __shfl_xor(sp, off);
    if (lane == 0) s_red[wave] = sp;
    lds_barrier();
    CSTAMP(9);
    if (tid == 0) {
        double s2 = 0.0;
        for (int w = 0; w < NT / 64; ++w) s2 += s_red[w];
        ctrl->spose_l[rung] = s2;
    }
}

template <int SOLVER, bool IMG>
__global__ __launch_bounds__(CT) void k_ctrl(lh_ctrl* __restrict__ ctrl, double* __restrict__ rs_commit,
                                             const double* __restrict__ rs_stage, const double* __restrict__ maxd_in,
                                             const uint16_t* __restrict__ pair_pq, const uint16_t* __restrict__ units,
                                             double* __restrict__ dxp, lh_params prm, int mode /* 0 init, 1 trial */,
                                             volatile int* __restrict__ host_done, int seq, double* __restrict__ img) {
    // S + lambda D (lower); L^T above, D in place; row NP = rhs -> z / D
    __shared__ __attribute__((aligned(16))) double A[(NP + 1) * AS];
    __shared__ __attribute__((aligned(16))) double dg[NP];   // the PCG's vector (16-byte reads)
    __shared__ double bpv[NP], hdv[NP], xs[NP];
    __shared__ uint16_t s_units[16 * LH_NSTEP];
    __shared__ int s_flags[4];
    __shared__ double s_red[CT / 64], s_lam;
    __shared__ __attribute__((aligned(16))) double s_pcg[48];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int P = prm.P, n = 6 * P, NE = (n + 15) & ~15;
    const lh_rs_layout LY = lh_rs_make(P, prm.npairs);
    // k_reduce took this trial's LM decision; a rung workgroup > 0 reads it (or workgroup 0's) from lh_ctrl
    const int rung = (int)blockIdx.x;
    const bool dec_src = mode != 0 && prm.dec_in_reduce;
    // A batch chain of a controller that decides itself (sharded: after the exchange) is decided by the launch's
    // last workgroup (lh_launch_ctrl adds it), and every other workgroup, 0 included, waits for that decision
    // (this chain's evo word: no decision has rewritten it yet)
    const int nwg = prm.ladder > 1 ? prm.ladder : 1;
    const bool dwg = !dec_src && mode != 0;   // the decider workgroup decides this chain
    if (!prm.dec_in_reduce && rung == nwg) {
        if (dwg && threadIdx.x == 0)
            ctrl_decider(ctrl, prm, rs_stage, LY, __builtin_amdgcn_readfirstlane(ctrl->evo) >> 8, host_done, seq);
        return;
    }
    const bool decided = dec_src || rung > 0 || dwg;
    const bool nd = SOLVER == 0 && prm.nd_steps > 0;        // the two-chain LDL^T schedule
    // k_reduce wrote S and b_s in this kernel's LDS layout (img[0] staged, img[1] committed): the system
    // arrives by a straight copy, no index math per entry (the scatter below was 2.2 us of wave 0's time)
    constexpr bool imgp = IMG;   // (the host sets prm.img only for SOLVER 0 without the two-chain schedule)
    static_assert(AS == LH_IMG_AS && (NP + 1) * AS == LH_IMG_SZ && LH_IMG_SZ % 2 == 0, "k_reduce's image layout");
    // the image is copied by waves 1-15 (wave 0 factors block 0 meanwhile): copy thread ctid = tid - 64 takes the
    // double pairs ctid + CW u
    constexpr int CW = CT - 64, IMG2 = LH_IMG_SZ / 2, NIMG = (IMG2 + CW - 1) / CW;
    const int ctid = tid - 64;
    const bool cpw = tid >= 64;
#ifdef LH_STAMPS
    const unsigned long long ct_start = __builtin_amdgcn_s_memtime(), rt_start = __builtin_amdgcn_s_memrealtime();
    // [160 + wave]: the wave's HW_ID word (SIMD in bits 5:4): which waves share wave 0's SIMD
    if (lane == 0) lh_stamps[160 + wave] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) | (1ull << 32);
#endif

    // ---------------- 1. prefetch (one round trip) ----------------
    double tchi = 0.0, sl = 0.0, ndg = 0.0;
    CtrlWords cw{};
    if (!decided && tid == 0) {
        cw = ctrl_load(ctrl);
        tchi = 0.5 * rs_stage[LY.off_sc + LH_SC_CHI2];
        sl = rs_stage[LY.off_sc + LH_SC_SCALE];
        ndg = rs_stage[LY.off_sc + LH_SC_NDEG];
    }
    // the decision's words: uniform loads in the same round trip as the system
    int done = 0, accept = 0, skip = 0;
    double lambda = 0.0;
    int dseq = -1;
    bool staged_is_commit = false;   // an evaluate-only trial: k_reduce copied the committed system to the staged side
    // workgroup `rung` > 0 of a ladder launch: the same system at the lambda of the rung-th rejection
#ifdef LH_STAMPS
    if (rung) return;   // (the diagnostic build times one controller)
#endif
    // (the initial linearisation's controller builds no ladder: its release on workgroup 0's path cost ~5 us per
    // solve, and a rejection right after it refactors and builds one)
    if (rung && mode == 0) return;
    // the decider workgroup decides and publishes (workgroup 0's thread 0 below decides the initial linearisation)
    if (dwg) ladder_wait(ctrl, seq);
    if (decided) {
        const LadderDec d = ladder_read(ctrl, prm, seq, rung);   // (the rung's lambda: block 0's early factor uses it)
        done = d.done;
        accept = d.accept;
        skip = d.skip;
        lambda = d.lambda;
        dseq = __builtin_amdgcn_readfirstlane(ctrl->done_seq);
        staged_is_commit = imgp && __builtin_amdgcn_readfirstlane(ctrl->evo_seq[seq & 1]) != 0;
    }
    // Round u covers elements [ER u, ER u + ER), thread t < ER element ER u + t (coalesced): its entry
    // (ea, eb) of a 6x6 S block is the same in every round and its block advances by 28, so the
    // element's rows need only the block's pose pair (p | q << 16, from the 840-byte pair table).
    // Only the staged system is loaded here: a trial is accepted far more often than not, and a
    // rejected one loads the committed system after the decision (one more round trip).
    const uint32_t* __restrict__ pqw = reinterpret_cast<const uint32_t*>(pair_pq);
    const int e36 = tid % 36, ea = e36 / 6, eb = e36 - 6 * ea, blk0 = tid / 36;
    const int ibase = (tid < ER) ? tid : (1 << 30);   // threads past ER hold no element
    double vs[NLD];
    uint32_t mp[NLD];
    double2 iv[NIMG];                   // imgp: this copy thread's double pairs ctid + CW u of the image
    double bpx = 0.0, hdx = 0.0;        // imgp: b_p and diag H_pp of row tid (the packed buffer)
    const double2* __restrict__ img2 = reinterpret_cast<const double2*>(img);
    // only the pairs that carry data are read (the lower triangle of the real rows and the rhs row: ~45 % of the
    // image at C3); the rest are zeros or the identity padding, written without a load (img_need, img_fill)
    auto img_need = [&](int k) {
        const int e = 2 * k, row = e / AS, col = e - AS * row;
        return k < IMG2 && ((row < n && col <= row) || (row == NP && col < n));
    };
    auto img_fill = [&](int k) {
        const int e = 2 * k, row = e / AS, col = e - AS * row;
        const bool pad = row >= n && row < NE;   // as k_img_init: identity on rows [n, NE)
        return double2{(pad && col == row) ? 1.0 : 0.0, (pad && col + 1 == row) ? 1.0 : 0.0};
    };
    if constexpr (imgp) {
        bpx = rs_stage[LY.off_bp + min(tid, n - 1)];
        hdx = rs_stage[LY.off_hd + min(tid, n - 1)];
    } else {
#pragma unroll
        for (int u = 0; u < NLD; ++u) {
            const int i = u * ER + ibase;
            vs[u] = (i < LY.total) ? rs_stage[i] : 0.0;
            mp[u] = pqw[min(blk0 + (ER / 36) * u, max(LY.npairs - 1, 0))];
        }
    }
    uint32_t unit2 = 0;   // two unit words per thread (SOLVER 0)
    if (SOLVER == 0 && tid < 8 * LH_NSTEP) unit2 = reinterpret_cast<const uint32_t*>(units)[tid];
    // The one-chain LDL^T's first block (rows 0-7: pose 0 and two rows of pose 1) is factored by wave 0
    // while the other waves scatter: its row r = lane & 7 comes straight from the packed pair blocks
    // (pairs (0, 0), (0, 1), (1, 1) at indices 0, 1, P: every pair is listed for P <= LH_PMAX), staged
    // and committed, selected once the decision is known; the scatter leaves block 0 alone.
    const bool early0 = SOLVER == 0 && !(prm.nd_steps > 0) && n >= 8;
    double b0s[8], b0c[8];
    if (imgp && early0 && wave == 0) {   // rows 0-7 of the staged image (the upper entries are zeros, unused)
        const int r = lane & 7;
#pragma unroll
        for (int q = 0; q < 8; ++q) b0s[q] = img[r * AS + q];
    } else if (!imgp && early0 && wave == 0) {
        const int r = lane & 7;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            int i;
            if (r < 6 && q < 6) i = 6 * r + q;                           // pair (0, 0)
            else if (r >= 6 && q < 6) i = 36 + 6 * q + (r - 6);           // pair (0, 1): S(6 + eb, ea)
            else if (r < 6) i = 36 + 6 * r + (q - 6);                    // (upper, unused)
            else i = 36 * P + 6 * (r - 6) + (q - 6);                     // pair (1, 1)
            b0s[q] = rs_stage[i];
            b0c[q] = rs_commit[i];
        }
    }

    // imgp: the staged image goes into LDS as it arrives, before the decision is known (a trial is accepted
    // far more often than not; a rejected one overwrites it with the committed image); block 0 is wave 0's
    // (a macro, not a lambda: a captured array would live in scratch memory)
#define LH_IMG_TO_LDS()                                                                                        \
    do {                                                                                                       \
        double2* A2_ = reinterpret_cast<double2*>(A);                                                          \
        if (cpw) _Pragma("unroll") for (int u = 0; u < NIMG; ++u) {                                            \
            const int k = ctid + CW * u, e = 2 * k, row = e / AS, col = e - AS * row; /* AS even: no straddle */\
            if (k < IMG2 && !(early0 && row < 8 && col < 8)) A2_[k] = img_need(k) ? iv[u] : img_fill(k);      \
        }                                                                                                      \
    } while (0)
    // imgp with k_reduce's decision known: wave 0 factors block 0 first, while the image is still in flight (its
    // rows come in their own loads, b0s; the image copy leaves block 0 alone), then copies its share
    bool f0_done = false;
    if constexpr (imgp) {
    if (cpw) {   // wave-uniform: the copy waves' image loads and copy, apart from wave 0's factor (registers)
#pragma unroll
        for (int u = 0; u < NIMG; ++u) iv[u] = img2[img_need(ctid + CW * u) ? ctid + CW * u : 0];
        LH_IMG_TO_LDS();
    }
#ifndef LH_NO_F0_FIRST
    else if (early0 && decided && !done && !skip) {
        if (!accept && !staged_is_commit) {   // a rejected trial factors the committed block 0
            const int r = lane & 7;
#pragma unroll
            for (int q = 0; q < 8; ++q) b0s[q] = img[LH_IMG_SZ + r * AS + q];
        }
        const int r = lane & 7;
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            double x = b0s[q];
            if (q == r) x = (prm.strategy == 0) ? x + lambda : x + lambda * x;
            v[q] = x;
        }
        LdltBlockLds& F0 = ldlt_lds();
        factor_block8_v(LdsSys{A}, v, F0.N[0], F0.ND[0], 0, lane);
        f0_done = true;
    }
#endif
    }

    if (!decided) {
        if (mode == 0) {   // max |diag H_pp| for computeLambdaInitLM (problem.cpp:486-496)
            double mx = 0.0;
            if constexpr (imgp) {
                if (tid < n) mx = fabs(hdx);
            } else {
#pragma unroll
                for (int u = 0; u < NLD; ++u) {
                    const int i = u * ER + ibase;
                    if (i >= LY.off_hd && i < LY.off_hd + n) mx = fmax(mx, fabs(vs[u]));
                }
            }
            for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
            if (lane == 0) s_red[wave] = mx;
            lds_barrier();
        }
        // ---------------- LM bookkeeping (thread 0) ----------------
        if (tid == 0) {
            double mdiag = 0.0;
            if (mode == 0) {
                for (int w = 0; w < CT / 64; ++w) mdiag = fmax(mdiag, s_red[w]);
                mdiag = fmax(*maxd_in, mdiag);
            }
            int d_o, a_o, c_o;
            double lam_n;
            // (only the initial linearisation's: a later chain's is the decider workgroup's)
            s_flags[2] = ctrl_lm_step(ctrl, cw, prm, 0, mdiag, tchi, sl, ndg, host_done, seq, d_o, a_o, c_o, lam_n);
            s_flags[0] = d_o;
            s_flags[1] = a_o;
            s_lam = lam_n;
        }
        lds_barrier();
        done = s_flags[0];
        accept = s_flags[1];
        skip = s_flags[2];
        lambda = s_lam;
    }
    // this trial's k_reduce stopped the loop: the summary goes to the host and done is raised here
    if (dec_src && done && dseq == seq && tid == 0 && host_done && rung == 0) publish_stop(ctrl, host_done);
    if (done || skip) return;
    // the ladder: a factor builds prm.ladder rungs (every factor, or with ladder_eager off only one after a
    // rejection); rung r factors at the lambda r more rejections set, by ctrl_lm_step's own updates in its order
    const bool build = mode != 0 && ladder_build(prm, accept);
    if (rung != 0 && (!build || rung >= prm.ladder)) return;
    if (rung == 0 && tid == 0) ctrl->lad_n = build ? prm.ladder : 1;
    dxp += (size_t)rung * n;
#ifdef LH_STAMPS
    if (tid == 0) {
        atomicAdd(&lh_stamps[32], ct_start);
        atomicAdd(&lh_stamps[61], 1ull);
        atomicAdd(&lh_stamps[62], rt_start);
    }
#endif
    CSTAMP(1);
#ifdef LH_STAMPS
    if (tid == 0) __builtin_amdgcn_s_waitcnt(0);   // (diagnostic) thread 0's staged-system loads have arrived
#endif
    CSTAMP(2);

    // ---------------- 2. commit, diag + lambda, scatter into LDS (natural order) ----------------
    if constexpr (imgp) {
        // The image: a straight copy (16-byte LDS stores at consecutive addresses, issued above), lambda
        // added on the diagonal of the real rows by the thread that stored it (the identity padding and the
        // zero upper triangle come with the image).  k_reduce commits an accepted system to img[1] before
        // the next trial overwrites img[0] (commit_in_reduce's role), so nothing here copies S.  After an
        // evaluate-only trial the staged side already holds the committed system (k_reduce), so no reload.
        if (!accept && !staged_is_commit) {
            const double2* __restrict__ imgc2 = reinterpret_cast<const double2*>(img + LH_IMG_SZ);
#pragma unroll
            for (int u = 0; u < NIMG; ++u) iv[u] = imgc2[(cpw && img_need(ctid + CW * u)) ? ctid + CW * u : 0];
            bpx = rs_commit[LY.off_bp + min(tid, n - 1)];
            hdx = rs_commit[LY.off_hd + min(tid, n - 1)];
            if (early0 && wave == 0 && !f0_done) {
                const int r = lane & 7;
#pragma unroll
                for (int q = 0; q < 8; ++q) b0s[q] = img[LH_IMG_SZ + r * AS + q];
            }
            LH_IMG_TO_LDS();
        }
#undef LH_IMG_TO_LDS
#pragma unroll
        for (int u = 0; u < NIMG; ++u) {
            const int k = ctid + CW * u, e = 2 * k, row = e / AS, col = e - AS * row;
            if (cpw && k < IMG2 && row < n && (col == row || col + 1 == row) && !(early0 && row < 8)) {
                double& d = A[row * AS + row];
                d = (prm.strategy == 0) ? d + lambda : d + lambda * d;
            }
        }
        if (tid < n) {
            bpv[tid] = bpx;
            hdv[tid] = hdx;
        }
    } else {
    if (!accept) {   // rollback: the committed system, with the new lambda
#pragma unroll
        for (int u = 0; u < NLD; ++u) {
            const int i = u * ER + ibase;
            vs[u] = (i < LY.total) ? rs_commit[i] : 0.0;
        }
    }
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
        const int i = u * ER + ibase;
        const double v = vs[u];
        if (accept && rung == 0 && i < LY.total) rs_commit[i] = v;
        if (i < LY.off_bs) {
            // S element i: pose pair (p, q), p <= q, entry (ea, eb) -> rows 6 p + ea, 6 q + eb.  The
            // upper slot of every off-diagonal entry is zeroed: the factor stores L^T there where the
            // envelope reaches, and the back substitution reads zeros elsewhere.
            int pp = (int)(mp[u] & 0xffffu), qq = (int)(mp[u] >> 16);
            if (nd) {
                pp = lh_nd_pos(pp, P, prm.nd_a, prm.nd_s, prm.nd_long_first);
                qq = lh_nd_pos(qq, P, prm.nd_a, prm.nd_s, prm.nd_long_first);
            }
            const int gi = 6 * pp + ea, gj = 6 * qq + eb;
            const int hi = max(gi, gj), lo = min(gi, gj);
            if (early0 && hi < 8) {
                // block 0: wave 0's
            } else if (gi == gj) {
                A[gi * AS + gi] = (prm.strategy == 0) ? v + lambda : v + lambda * v;
            } else if (pp != qq || gi > gj) {
                A[hi * AS + lo] = v;
                A[lo * AS + hi] = 0.0;
            }
        } else if (i < LY.off_bp) {
            int r = i - LY.off_bs;
            if (nd) r = 6 * lh_nd_pos(r / 6, P, prm.nd_a, prm.nd_s, prm.nd_long_first) + r % 6;
            A[NP * AS + r] = v;
        } else if (i < LY.off_hd) {
            bpv[i - LY.off_bp] = v;
        } else if (i < LY.off_hd + n) {
            hdv[i - LY.off_hd] = v;
        }
    }
    if (tid >= n && tid < NE) {   // identity padding rows
        A[tid * AS + tid] = 1.0;
        A[NP * AS + tid] = 0.0;
    }
    for (int x = tid; x < (NE - n) * NE; x += CT) {
        const int r = n + x / NE, c = x - NE * (x / NE);
        if (c < r) {
            A[r * AS + c] = 0.0;
            A[c * AS + r] = 0.0;
        }
    }
    }   // packed path
    if (SOLVER == 0 && tid < 8 * LH_NSTEP) reinterpret_cast<uint32_t*>(s_units)[tid] = unit2;
    CSTAMP(3);
    if (early0 && wave == 0 && !f0_done) {
        const int r = lane & 7;
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            double x = (imgp || accept) ? b0s[q] : b0c[q];
            if (q == r) x = (prm.strategy == 0) ? x + lambda : x + lambda * x;
            v[q] = x;
        }
        LdltBlockLds& F = ldlt_lds();
        factor_block8_v(LdsSys{A}, v, F.N[0], F.ND[0], 0, lane);
    }
    lds_barrier();
    CSTAMP(4);

    // ---------------- 3-4. blocked LDL^T with the forward substitution in row NP; back substitution ----------------
    if constexpr (SOLVER == 1) {
        const int its = lds_pcg_solve(A, xs, dg, s_pcg, n, tid, prm.pcg_tol, (prm.pcg_max_it > 0 ? prm.pcg_max_it : 2 * n) + 1);
        if (tid == 0) {
            ctrl->lad_its[rung] = its;
            if (rung == 0) ctrl->pcg_iters += its;   // a higher rung's count is added when a rejection uses it
        }
    } else {
        if (nd) lds_ldlt_solve_nd(A, xs, n, tid, s_units, prm);
        else lds_ldlt_solve(A, xs, n, NE, tid, nullptr, s_units, LdltTail{ctrl, dxp, bpv, hdv, lambda, prm.strategy, rung},
                            early0);
    }
    CSTAMP(8);

    // the one-chain LDL^T took the tail in its back-substitution wave
    if (SOLVER == 1 || nd) ctrl_step_tail<CT>(ctrl, prm, n, lambda, xs, bpv, hdv, s_red, dxp, rung);
    CSTAMP(12);
#ifdef LH_STAMPS
    if (tid == 0) atomicAdd(&lh_stamps[63], (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
}

// ============================================================================
// k_ctrl_g: the controller for windows past LH_PMAX poses (21 < P <= LH_PMAX_WIN, 6P <= 384 rows).
// Same LM bookkeeping and pose tail as k_ctrl; the reduced system lives in global memory (gA,
// row-major, stride NG = ceil32(6P), L2-resident: <= 1.2 MB) instead of one CU's LDS.  Eigen's
// pivot order is the same static sort of |diag(S + lambda D)|.  The factorisation is a blocked
// right-looking LDL^T over 32-column panels:
//   (a) the panel (rows K.., columns K..K+31) into LDS;
//   (b) its 32x32 diagonal block by wave 0 in registers (lane r = row r; pivots and column
//       entries by lane broadcast);
//   (c) the panel rows below: one thread per row, 32 columns in registers;
//   (d) L and D back to gA;
//   (e) the trailing block, A_ij -= sum_k L_ik (D_k L_jk), as 16x16 f64 MFMA tiles (one wave per
//       tile, 8 MFMAs over the panel).
// Eigen semantics kept: a zero pivot skips the division (pivot_is_valid); if the largest |diag| is
// 0 there is no factorisation and the solves run on the raw matrix with identity transpositions.
// The triangular solves visit each row's terms in the oracle's order (ldlt_solve: ascending
// columns, 8-row panels whose zero entries skip in-panel updates; descending in L^T), so they
// are bitwise the oracle's solve of the same factor.  The factor's rounding differs from Eigen's
// left-looking dot products (parity to tolerance).
// ============================================================================
#define GNB 32                          // panel width
#define GNMAX (6 * LH_PMAX_WIN)         // largest reduced system
#define GPS (GNB + 1)                   // LDS panel row stride (conflict-free column reads)
#define GT 512                          // k_ctrl_g threads: 8 waves, 256 VGPRs (register rows in the factor)

// k_ctrl_g's reduced-system solve (shared with the probe): gA holds the permuted system's lower
// triangle (stride NG, identity padding to NG), yv the permuted right-hand side (LDS, n entries);
// on return yv holds the solution in pivot order and gA the factor.  All CT threads.
__device__ __forceinline__ void g_ldlt_solve(double* __restrict__ gA, int NG, int n, bool all_zero, double* yv,
                                             double* pnl) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ double ginv[GNB];   // 1/D of the current block's pivots (1 where the pivot is invalid)
    __shared__ double gdia[GNB];   // D of the current block's pivots
    CSTAMP(5);
    // ---------------- blocked right-looking LDL^T ----------------
    if (!all_zero) {
        for (int K = 0; K < NG; K += GNB) {
            const int m = NG - K;
            // (a) the panel into LDS (lower part of the diagonal block, all of the rows below)
            for (int x = tid; x < m * GNB; x += GT) {
                const int r = x / GNB, c = x - GNB * (x / GNB);
                pnl[r * GPS + c] = (r >= c) ? gA[(size_t)(K + r) * NG + K + c] : 0.0;
            }
            lds_barrier();
            CSTAMP(13);
            // (b) the diagonal block: wave 0, lane j holds column j of the full symmetric block in
            //     registers (c[i] = A(i, j)).  Step k: D_k and the column k entries come from lane k
            //     by readlane (uniform values); lane j's own L(j, k) is its register c[k] (the
            //     symmetric copy), so nothing is indexed per lane and nothing goes through memory.
            if (wave == 0) {
                const int j = lane & (GNB - 1);
                double c[GNB];
#pragma unroll
                for (int i = 0; i < GNB; ++i) c[i] = (i >= j) ? pnl[i * GPS + j] : pnl[j * GPS + i];
#pragma unroll
                for (int k = 0; k < GNB; ++k) {
                    const double d = readlane_d(c[k], k);
                    const double id = (fabs(d) > 0.0) ? fast_rcp(d) : 1.0;   // pivot_is_valid: no division
                    const double wj = d * (c[k] * id);                        // D_k L(j, k)
#pragma unroll
                    for (int i = k + 1; i < GNB; ++i) {
                        const double lik = readlane_d(c[i], k) * id;          // L(i, k), uniform
                        c[i] -= lik * wj;
                    }
                    // row j of column k becomes L(j, k) for j > k; lanes j <= k scale entries they never
                    // read again (the diagonal D_k is kept in gdia), so no lane masks are needed
                    c[k] *= id;
                    if (lane == 0) { ginv[k] = id; gdia[k] = d; }
                }
                // lane j ends with row j of the factor: c[i] = L(j, i) for i < j (its symmetric copies,
                // scaled at step i); the rest of its row is written too (the upper part is overwritten
                // by (c), the diagonal below)
                if (lane < GNB) {
#pragma unroll
                    for (int i = 0; i < GNB; ++i) pnl[j * GPS + i] = c[i];
                }
                wave_sync();
                if (lane < GNB) pnl[lane * GPS + lane] = gdia[lane];
            }
            lds_barrier();
            CSTAMP(14);
            // (c) the panel rows below the block.  W = D_k L(j, k) (j > k) into the diagonal block's
            //     free upper triangle; each row in registers, right-looking: the same operations and
            //     roundings as the diagonal block's rows.
            if (wave == 0 && lane < GNB)
                for (int j = lane + 1; j < GNB; ++j) pnl[lane * GPS + j] = pnl[lane * GPS + lane] * pnl[j * GPS + lane];
            lds_barrier();
            // the W rows' LDS addresses off an opaque zero: one base register and immediate offsets (with
            // constant addresses the compiler kept ~160 of them in VGPRs across the loop, and spilled)
            int z0 = 0;
            asm volatile("" : "+v"(z0));
            for (int r = GNB + tid; r < m; r += GT) {
                double a[GNB];
#pragma unroll
                for (int c = 0; c < GNB; ++c) a[c] = pnl[r * GPS + c];
#pragma unroll
                for (int k = 0; k < GNB; ++k) {
                    const double l = a[k] * ginv[k];
                    a[k] = l;
#pragma unroll
                    for (int j = k + 1; j < GNB; ++j) a[j] -= l * pnl[z0 + k * GPS + j];
                    __builtin_amdgcn_sched_barrier(0);   // one step's loads at a time (register budget)
                }
#pragma unroll
                for (int c = 0; c < GNB; ++c) pnl[r * GPS + c] = a[c];
            }
            lds_barrier();
            CSTAMP(15);
            // (d) L and D of the panel back to gA
            for (int x = tid; x < m * GNB; x += GT) {
                const int r = x / GNB, c = x - GNB * (x / GNB);
                if (r >= c) gA[(size_t)(K + r) * NG + K + c] = pnl[r * GPS + c];
            }
            // (e) trailing block: 16x16 tiles (I >= J), four per wave at a time (their loads in flight
            //     together), 8 f64 MFMAs per tile over the panel
            const int mt = (m - GNB) >> 4;
            const int ntiles = mt * (mt + 1) / 2;
            for (int t0 = 4 * wave; t0 < ntiles; t0 += 4 * (GT / 64)) {
                int I[4], J[4];
                v4d acc[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int t = min(t0 + u, ntiles - 1);
                    int ii = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
                    while ((ii + 1) * (ii + 2) / 2 <= t) ++ii;
                    while (ii * (ii + 1) / 2 > t) --ii;
                    I[u] = ii;
                    J[u] = t - ii * (ii + 1) / 2;
                    const int r0 = K + GNB + 16 * I[u], c0 = K + GNB + 16 * J[u];
#pragma unroll
                    for (int v = 0; v < 4; ++v) acc[u][v] = gA[(size_t)(r0 + (lane >> 4) + 4 * v) * NG + c0 + (lane & 15)];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
#pragma unroll
                    for (int kk = 0; kk < GNB; kk += 4) {
                        const int k = kk + (lane >> 4);
                        const double av = -pnl[(GNB + 16 * I[u] + (lane & 15)) * GPS + k];
                        const double bv = pnl[k * GPS + k] * pnl[(GNB + 16 * J[u] + (lane & 15)) * GPS + k];
                        acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[u], 0, 0, 0);
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (t0 + u >= ntiles) break;
                    const int r0 = K + GNB + 16 * I[u], c0 = K + GNB + 16 * J[u];
#pragma unroll
                    for (int v = 0; v < 4; ++v) gA[(size_t)(r0 + (lane >> 4) + 4 * v) * NG + c0 + (lane & 15)] = acc[u][v];
                }
            }
            __syncthreads();
            CSTAMP(16);
        }
    }

    CSTAMP(6);
    // the factor's diagonal blocks into LDS (the panel buffer is free now): block b's rows at
    // pnl[(32 b + r) * GPS + c], one round trip for all of them
    for (int x = tid; x < n * GNB; x += GT) {
        const int r = x / GNB, c = x - GNB * (x / GNB);
        const int K = r & ~(GNB - 1);
        pnl[r * GPS + c] = (K + c < n) ? gA[(size_t)r * NG + K + c] : 0.0;
    }
    lds_barrier();
    // ---------------- forward substitution (unit L), the oracle's order ----------------
    static_assert(GNMAX <= GT, "one row per thread in the solves' row updates");
    for (int K = 0; K < n; K += GNB) {
        const int kb = min(GNB, n - K);
        // the block's columns of the rows below: loaded first (they do not depend on the solve), so
        // their latency overlaps the diagonal block's chain
        const int ib = K + kb + tid;
        double Lb[GNB];
#pragma unroll
        for (int k = 0; k < GNB; ++k) Lb[k] = (ib < n && k < kb) ? gA[(size_t)ib * NG + K + k] : 0.0;
        if (wave == 0) {
            const int r = lane & (GNB - 1);
            double x = yv[K + r];
            double Lr[GNB];
#pragma unroll
            for (int k = 0; k < GNB; ++k) Lr[k] = (r > k && K + r < n) ? pnl[(K + r) * GPS + k] : 0.0;
#pragma unroll
            for (int k = 0; k < GNB; ++k) {
                const double xk = readlane_d(x, k);   // uniform: an SGPR pair, no LDS round trip
                if (k < kb && r > k && r < kb) {
                    const bool same_panel = (r >> 3) == (k >> 3);
                    if (!same_panel || xk != 0.0) x -= Lr[k] * xk;
                }
            }
            if (lane < kb) yv[K + lane] = x;
        }
        lds_barrier();
        if (ib < n) {   // the block's columns, ascending
            double x = yv[ib];
#pragma unroll
            for (int k = 0; k < GNB; ++k)
                if (k < kb) x -= Lb[k] * yv[K + k];
            yv[ib] = x;
        }
        lds_barrier();
    }
    // D^+ (tolerance: numeric_limits<double>::min())
    for (int i = tid; i < n; i += GT) {
        const double d = pnl[i * GPS + (i & (GNB - 1))];
        yv[i] = (fabs(d) > 2.2250738585072014e-308) ? yv[i] / d : 0.0;
    }
    lds_barrier();
    // ---------------- back substitution (L^T), descending ----------------
    for (int K = ((n - 1) / GNB) * GNB; K >= 0; K -= GNB) {
        const int kb = min(GNB, n - K);
        const int ia = tid;   // the rows above the block: their L^T entries, loaded ahead as above
        double La[GNB];
#pragma unroll
        for (int k = 0; k < GNB; ++k) La[k] = (ia < K && k < kb) ? gA[(size_t)(K + k) * NG + ia] : 0.0;
        if (wave == 0) {
            const int r = lane & (GNB - 1);
            double x = yv[K + r];
            double Lc[GNB];
#pragma unroll
            for (int k = 0; k < GNB; ++k) Lc[k] = (k > r && k < kb) ? pnl[(K + k) * GPS + r] : 0.0;
#pragma unroll
            for (int k = GNB - 1; k >= 0; --k) {
                const double xk = readlane_d(x, k);
                if (k < kb && r < k) x -= Lc[k] * xk;
            }
            if (lane < kb) yv[K + lane] = x;
        }
        lds_barrier();
        if (ia < K) {   // the block's rows, descending
            double x = yv[ia];
#pragma unroll
            for (int k = GNB - 1; k >= 0; --k)
                if (k < kb) x -= La[k] * yv[K + k];
            yv[ia] = x;
        }
        lds_barrier();
    }
    CSTAMP(7);
}

// k_dense: the reduced system's S blocks (packed per pose pair, p <= q) into the dense symmetric n x n
// matrix gS[1 - cur] (stride NG) that k_ctrl_g gathers from in pivot order.  One 64-thread block per
// pair, launched after the exchange (when there is one) and before k_ctrl_g; gS is double-buffered
// with the committed state (ctrl->cur), so a rejected trial keeps the committed copy.
__global__ __launch_bounds__(64) void k_dense(const double* __restrict__ rs, const uint16_t* __restrict__ pair_pq,
                                              const lh_ctrl* __restrict__ ctrl, double* __restrict__ gS, int P, int NG) {
    const int done = __builtin_amdgcn_readfirstlane(ctrl->done);
    const int evo = __builtin_amdgcn_readfirstlane(ctrl->evo);   // k_reduce wrote no S blocks
    const int cur = __builtin_amdgcn_readfirstlane(ctrl->cur);
    if (done || evo) return;
    const lh_rs_layout LY = lh_rs_make(P, P * (P + 1) / 2);   // the dense packed layout (P <= LH_PMAX_WIN)
    const int b = blockIdx.x, lane = threadIdx.x;
    const int p = pair_pq[2 * b], q = pair_pq[2 * b + 1];
    if (lane >= 36) return;
    const int a = lane / 6, c = lane - 6 * (lane / 6);
    const double v = rs[LY.off_S + b * 36 + lane];
    double* g = gS + (size_t)(1 - cur) * NG * NG;
    g[(size_t)(6 * p + a) * NG + 6 * q + c] = v;
    if (p != q) g[(size_t)(6 * q + c) * NG + 6 * p + a] = v;   // a diagonal block has both halves already
}

__global__ __launch_bounds__(GT) void k_ctrl_g(lh_ctrl* __restrict__ ctrl, double* __restrict__ rs_commit,
                                               const double* __restrict__ rs_stage, const double* __restrict__ maxd_in,
                                               const uint32_t* __restrict__ rsmap,
                                               double* __restrict__ dxp, lh_params prm, int mode,
                                               volatile int* __restrict__ host_done, int seq, double* __restrict__ gA,
                                               const double* __restrict__ gS) {
    __shared__ double pnl[GNMAX * GPS];
    __shared__ double dg[GNMAX], bsv[GNMAX], bpv[GNMAX], hdv[GNMAX], xs[GNMAX], yv[GNMAX], gkey[GNMAX];
    __shared__ int perm[GNMAX], iperm[GNMAX];
    __shared__ int s_flags[4];
    __shared__ double s_red[GT / 64], s_lam;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int P = prm.P, n = 6 * P, NG = (n + GNB - 1) & ~(GNB - 1);
    const lh_rs_layout LY = lh_rs_make(P, prm.npairs);
#ifdef LH_STAMPS
    const unsigned long long ct_start = __builtin_amdgcn_s_memtime(), rt_start = __builtin_amdgcn_s_memrealtime();
#endif

    // ---------------- controller words, pose matrices, max |diag| (mode 0) ----------------
    // workgroup `rung` > 0: a lambda-ladder rung with its own gA; it waits for workgroup 0's decision
    const int rung = (int)blockIdx.x;
#ifdef LH_STAMPS
    if (rung) return;
#endif
    if (rung && mode == 0) return;   // (the initial linearisation builds no ladder, as k_ctrl)
    if (rung) {
        ladder_wait(ctrl, seq);
        const LadderDec d = ladder_read(ctrl, prm, seq, rung);
        if (tid == 0) {
            s_flags[0] = d.done;
            s_flags[1] = d.accept;
            s_flags[2] = ctrl->cur;
            s_flags[3] = d.skip;
            s_lam = d.lambda;
        }
        lds_barrier();
    }
    double tchi = 0.0, sl = 0.0, ndg = 0.0;
    CtrlWords cw{};
    if (tid == 0 && !rung) {
        cw = ctrl_load(ctrl);
        tchi = 0.5 * rs_stage[LY.off_sc + LH_SC_CHI2];
        sl = rs_stage[LY.off_sc + LH_SC_SCALE];
        ndg = rs_stage[LY.off_sc + LH_SC_NDEG];
    }
    if (!rung) {
        double mx = 0.0;
        if (mode == 0)
            for (int i = tid; i < n; i += GT) mx = fmax(mx, fabs(rs_stage[LY.off_hd + i]));
        for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
        if (lane == 0) s_red[wave] = mx;
    }
    lds_barrier();
    if (tid == 0 && !rung) {
        double mdiag = 0.0;
        if (mode == 0) {
            for (int w = 0; w < GT / 64; ++w) mdiag = fmax(mdiag, s_red[w]);
            mdiag = fmax(*maxd_in, mdiag);
        }
        int done, accept, cur;
        double lam_n;
        __shared__ int b_cnt[4];
        s_flags[3] = ctrl_decide(ctrl, cw, prm, mode, mdiag, tchi, sl, ndg, rs_stage, LY, host_done, seq, done, accept, cur,
                                 lam_n, b_cnt);
        if (prm.ladder > 1 && mode != 0) ladder_publish(ctrl, seq);   // the rung workgroups wait for it
        s_flags[0] = done;
        s_flags[1] = accept;
        s_flags[2] = cur;
        s_lam = lam_n;
    }
    lds_barrier();
    const int done = s_flags[0], accept = s_flags[1], cur = s_flags[2];
    if (done || s_flags[3]) return;   // stopped, an evaluate-only acceptance, or a rejection onto a built rung
    const double lambda = s_lam;
    {
        const bool build = mode != 0 && ladder_build(prm, accept);
        if (rung != 0 && (!build || rung >= prm.ladder)) return;
        if (rung == 0 && tid == 0) ctrl->lad_n = build ? prm.ladder : 1;
        gA += (size_t)rung * prm.lad_stride;
        dxp += (size_t)rung * n;
    }

#ifdef LH_STAMPS
    if (tid == 0) {
        atomicAdd(&lh_stamps[32], ct_start);
        atomicAdd(&lh_stamps[61], 1ull);
        atomicAdd(&lh_stamps[62], rt_start);
    }
#endif
    CSTAMP(1);

    // ---------------- diagonal + lambda and right-hand sides (one round trip) ----------------
    // S of the chosen system is k_dense's dense copy gS[cur] (cur after the decision: the candidate's
    // on accept, the committed one on reject); the right-hand sides come from the packed system.
    const double* __restrict__ src = accept ? rs_stage : rs_commit;
    const double* __restrict__ gSc = gS + (size_t)cur * NG * NG;
    for (int i = tid; i < n; i += GT) {
        const double v = gSc[(size_t)i * NG + i];
        dg[i] = (prm.strategy == 0) ? v + lambda : v + lambda * v;
        bsv[i] = src[LY.off_bs + i];
        bpv[i] = src[LY.off_bp + i];
        hdv[i] = src[LY.off_hd + i];
    }
    lds_barrier();
    CSTAMP(2);

    // ---------------- pivot order: |diag| descending, ties by index, NaN last (as k_ctrl) ----------------
    for (int i = tid; i < n; i += GT) {   // the sort keys once
        const double d = fabs(dg[i]);
        gkey[i] = (d == d) ? d : -1.0;
    }
    lds_barrier();
    for (int row = tid; row < n; row += GT) {
        const double di = gkey[row];
        int r = 0;
#pragma unroll 8
        for (int j = 0; j < n; ++j) {
            const double d = gkey[j];
            r += (d > di) || (d == di && j < row);
        }
        perm[r] = row;
        iperm[row] = r;
    }
    lds_barrier();
    // Eigen's k = 0 test: the largest |diag| is not > 0 -> identity transpositions, no factorisation
    const bool all_zero = !(fabs(dg[perm[0]]) > 0.0);
    lds_barrier();
    if (all_zero)
        for (int i = tid; i < n; i += GT) { perm[i] = i; iperm[i] = i; }
    lds_barrier();
    CSTAMP(3);

    // ---------------- commit (the packed right-hand sides), gather gA (permuted lower triangle) ----------------
    // S itself is double-buffered as gS (the decision picked the buffer): only the part after it commits
    if (accept && rung == 0)
        for (int i = LY.off_bs + tid; i < LY.total; i += GT) rs_commit[i] = src[i];
    // gA(r, c) = S(perm r, perm c), r > c: a wave per row (lanes over columns), so its stores are
    // contiguous and its loads fall in one row of gS; eight rows per wave at a time, 48 loads in flight
    static_assert(GNMAX <= 6 * 64, "six 64-column chunks cover a row");
    for (int r0 = wave; r0 < NG; r0 += 8 * (GT / 64)) {
        double v[8][6];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int r = r0 + u * (GT / 64);
            const int pr = (r < n) ? perm[r] : 0;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const int c = 64 * j + lane;
                v[u][j] = (c < r && r < n) ? gSc[(size_t)pr * NG + perm[c]] : 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int r = r0 + u * (GT / 64);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const int c = 64 * j + lane;
                if (c < r && r < NG) gA[(size_t)r * NG + c] = v[u][j];
            }
        }
    }
    for (int i = tid; i < NG; i += GT) {
        gA[(size_t)i * NG + i] = i < n ? dg[perm[i]] : 1.0;
        yv[i] = i < n ? bsv[perm[i]] : 0.0;
    }
    __syncthreads();   // global stores before the panel loads
    CSTAMP(4);
    g_ldlt_solve(gA, NG, n, all_zero, yv, pnl);
    for (int i = tid; i < n; i += GT) { xs[perm[i]] = yv[i]; dxp[perm[i]] = yv[i]; }
    lds_barrier();
    CSTAMP(8);
    ctrl_step_tail<GT>(ctrl, prm, n, lambda, xs, bpv, hdv, s_red, nullptr, rung);
    CSTAMP(12);
#ifdef LH_STAMPS
    if (tid == 0) atomicAdd(&lh_stamps[63], (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
}

// ============================================================================
// k_ctrl_b: the controller for windows past LH_PMAX poses whose reduced system is banded (the
// reference's live solver, LDL^T, problem.cpp:420, at any window size).  In
// natural pose order a sliding window's S is block-banded: a landmark couples the poses of its run
// of keyframes, so row r's nonzeros start at its envelope fc(r) >= r - 104 (the host checks this per
// window, lh_host.cpp; other windows go to k_ctrl_g or PCG).  The blocked LDL^T of k_ctrl then needs
// only 8 tile rows (128 rows) of S at a time: the window holds them in one CU's LDS as a circular
// buffer (BandSys), and waves 12-15 stream the next tile row in, written into the slots of the tile row
// that just retired: one rank reads it from the band image k_reduce wrote in the loaders' order (prm.bimg,
// two steps ahead); a sharded solve from the all-reduced packed blocks (block indices two steps ahead,
// values one step ahead).  L goes
// to global memory row by row, ND per block; the back substitution (one wave) reads them back.  The
// per-step work units come from the same envelope (lh_ctrl_units over 11 unit waves).  One 1024-thread
// workgroup; the LM bookkeeping is k_reduce's (dec_in_reduce: one rank) or thread 0's (the initial
// linearisation); k_reduce also commits accepted systems (commit_in_reduce), so nothing here copies S.
// ============================================================================
template <bool B> struct BoolTag { static constexpr bool value = B; };
#define BNMAX (6 * LH_PMAX_ANY)         // largest reduced system (1536 rows)
#define BSTEP_MAX (BNMAX / 8)           // LDL^T steps
// the stream loaders: waves 12-15 (moving them off wave 0's SIMD, to 11 and 13-15, measured slower: the
// wave forming z then set the step); z and the ND copy are wave LH_BZW's (below)
__device__ __forceinline__ bool band_loader(int w) { return w >= 12; }
__device__ __forceinline__ int band_loader_slot(int w) { return w - 12; }
#ifndef LH_BZW
#define LH_BZW 8   // the wave that forms z and copies ND out: a unit wave idle in most steps (wave 12, a loader:
                    // P = 128 0.2113 against 0.2104 ms per trial, profiles/r05l_band_ab_bzw8.txt)
#endif
#define BZW LH_BZW

// S(r, c), c <= r < n, of the packed system: block (pose(c), pose(r)) through the per-window table
// bblk[p * 64 + d] (the block of pose pair (p, p + d), -1 where no chunk couples them)
__device__ __forceinline__ int band_block(const int32_t* __restrict__ bblk, int r, int c, int n) {
    const int pc = c / 6, pr = r / 6, d = pr - pc;
    return (c <= r && r < n && d < 64) ? bblk[pc * 64 + d] : -1;
}
__device__ __forceinline__ double band_value(const double* __restrict__ src, int blk, int r, int c, double lambda,
                                             int strategy, int n) {
    double v = (blk >= 0) ? src[(size_t)blk * 36 + (c % 6) * 6 + (r % 6)] : 0.0;
    if (r == c) {
        if (r >= n) v = 1.0;   // identity padding
        else v = (strategy == 0) ? v + lambda : v + lambda * v;
    }
    return v;
}

// LU: some step needs more than the 11 unit waves (chunk windows of ~16 poses), so the stream loaders take units
// too (a separate instantiation: the loaders' unit path costs ~1 % where no step needs it)
template <bool LU>
__global__ __launch_bounds__(CT) void k_ctrl_b(lh_ctrl* __restrict__ ctrl, const double* __restrict__ rs_commit,
                                               const double* __restrict__ rs_stage, const double* __restrict__ maxd_in,
                                               const int32_t* __restrict__ bblk, const uint16_t* __restrict__ bunits,
                                               double* __restrict__ Lg, double* __restrict__ NDg, double* __restrict__ dxp,
                                               lh_params prm, int mode, volatile int* __restrict__ host_done, int seq,
                                               const double* __restrict__ bimg) {
    __shared__ __attribute__((aligned(16))) double A[128 * AS];   // the circular window of the lower band
    __shared__ __attribute__((aligned(16))) double y[BNMAX];   // rhs (forward substitution), then x
    __shared__ double z[BNMAX];                             // D^-1 L^-1 b
    __shared__ __attribute__((aligned(16))) double Nl[2][64], NDl[2][64];
    __shared__ int s_flags[4];
    __shared__ double s_red[CT / 64], s_lam;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const int P = prm.P, n = 6 * P, NE = (n + 15) & ~15, nb = (n + 7) & ~7, NT = NE / 16, nstep = nb / 8;
    const lh_rs_layout LY = lh_rs_make(P, prm.npairs);
    // workgroup `rung` > 0: a lambda-ladder rung (k_ctrl's scheme), with its own L rows and ND
    const int rung = (int)blockIdx.x;
    const bool dec_src = mode != 0 && prm.dec_in_reduce;
    const bool decided = dec_src || rung > 0;
#ifdef LH_STAMPS
    const unsigned long long ct_start = __builtin_amdgcn_s_memtime(), rt_start = __builtin_amdgcn_s_memrealtime();
#endif
    // ---------------- the decision ----------------
    int done = 0, accept = 0, skip = 0;
    double lambda = 0.0;
#ifdef LH_STAMPS
    if (rung) return;
#endif
    if (rung && mode == 0) return;   // (the initial linearisation builds no ladder, as k_ctrl)
    if (rung && !dec_src) ladder_wait(ctrl, seq);   // workgroup 0 decides and publishes
    if (decided) {
        const LadderDec d = ladder_read(ctrl, prm, seq, rung);
        done = d.done;
        accept = d.accept;
        skip = d.skip;
        lambda = d.lambda;
        // this trial's k_reduce stopped the loop: the host's done is raised here (ctrl_lm_step)
        if (dec_src && done && tid == 0 && host_done && ctrl->done_seq == seq && rung == 0) publish_stop(ctrl, host_done);
    } else {
        double tchi = 0.0, sl = 0.0, ndg = 0.0;
        CtrlWords cw{};
        if (tid == 0) {
            cw = ctrl_load(ctrl);
            tchi = 0.5 * rs_stage[LY.off_sc + LH_SC_CHI2];
            sl = rs_stage[LY.off_sc + LH_SC_SCALE];
            ndg = rs_stage[LY.off_sc + LH_SC_NDEG];
        }
        double mx = 0.0;
        if (mode == 0)
            for (int i = tid; i < n; i += CT) mx = fmax(mx, fabs(rs_stage[LY.off_hd + i]));
        for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
        if (lane == 0) s_red[wave] = mx;
        lds_barrier();
        if (tid == 0) {
            double mdiag = 0.0;
            if (mode == 0) {
                for (int w = 0; w < CT / 64; ++w) mdiag = fmax(mdiag, s_red[w]);
                mdiag = fmax(*maxd_in, mdiag);
            }
            int d_o, a_o, c_o;
            double lam_n;
            __shared__ int b_cnt[4];
            s_flags[2] = ctrl_decide(ctrl, cw, prm, mode, mdiag, tchi, sl, ndg, rs_stage, LY, host_done, seq, d_o, a_o, c_o,
                                     lam_n, b_cnt);
            if (prm.ladder > 1 && mode != 0) ladder_publish(ctrl, seq);   // the rung workgroups wait for it
            s_flags[0] = d_o;
            s_flags[1] = a_o;
            s_lam = lam_n;
        }
        lds_barrier();
        done = s_flags[0];
        accept = s_flags[1];
        skip = s_flags[2];
        lambda = s_lam;
    }
    if (done || skip) return;
    {
        const bool build = mode != 0 && ladder_build(prm, accept);
        if (rung != 0 && (!build || rung >= prm.ladder)) return;
        if (rung == 0 && tid == 0) ctrl->lad_n = build ? prm.ladder : 1;
        const size_t NEs = (size_t)NE;
        Lg += (size_t)rung * (NEs * LH_LBW + (size_t)BSTEP_MAX * 64);   // lh_band_args: per rung, L rows | ND
        NDg += (size_t)rung * (NEs * LH_LBW + (size_t)BSTEP_MAX * 64);
        dxp += (size_t)rung * n;
    }
#ifdef LH_STAMPS
    if (tid == 0) {
        atomicAdd(&lh_stamps[32], ct_start);
        atomicAdd(&lh_stamps[61], 1ull);
        atomicAdd(&lh_stamps[62], rt_start);
    }
#endif
    CSTAMP(1);
    const double* __restrict__ src = accept ? rs_stage : rs_commit;
    // prm.bimg: k_reduce wrote the band in the loaders' order (lh_bimg_idx; staged, then committed): one load per
    // element, no block-index round trip before it
    const bool bim = prm.bimg != 0;
    const double* __restrict__ bsrc = bimg + (accept ? 0 : (size_t)NT * LH_BIMG_TR);

    // ---------------- the rhs, the first 8 tile rows, this wave's unit words ----------------
    for (int i = tid; i < NE; i += CT) {
        y[i] = (i < n) ? src[LY.off_bs + i] : 0.0;
        z[i] = 0.0;
    }
    {
        // 16 elements of the first window per thread: element k at row 8 k + tid / 128, column tid mod 128, so a
        // wave's writes go to consecutive columns (one row of 16-column stripes per thread put 8 lanes of a
        // 16-lane write group on one bank pair)
        constexpr int PER = 128 * 128 / CT;
        const int c0 = tid & 127, rr = tid >> 7;
        int bk[PER];
        if (bim) {
            double bv[PER];
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const int r = 8 * k + rr;
                bv[k] = (r < NE && c0 <= r) ? bsrc[lh_bimg_idx(r, c0)] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const int r = 8 * k + rr;
                double v = bv[k];
                if (r == c0) v = (r >= n) ? 1.0 : ((prm.strategy == 0) ? v + lambda : v + lambda * v);
                A[r * AS + c0] = v;
            }
        } else {
#pragma unroll
            for (int k = 0; k < PER; ++k) bk[k] = band_block(bblk, 8 * k + rr, c0, n);
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const int r = 8 * k + rr;
                A[r * AS + c0] = (r < NE && c0 <= r) ? band_value(src, bk[k], r, c0, lambda, prm.strategy, n) : 0.0;
            }
        }
    }
    uint32_t uwa = 0, uwb = 0;   // this wave's unit words: steps 2j, 2j + 1 in u32 j (lane j, lane j + 64)
    {
        const uint32_t* uw32 = reinterpret_cast<const uint32_t*>(bunits + (size_t)wv * BSTEP_MAX);
        uwa = uw32[lane];
        if (lane + 64 < BSTEP_MAX / 2) uwb = uw32[lane + 64];
    }
    auto unit_word = [&](int t) -> uint32_t {
        const int j = t >> 1;
        const uint32_t w = (j < 64) ? __builtin_amdgcn_readlane(uwa, j & 63) : __builtin_amdgcn_readlane(uwb, j & 63);
        return (t & 1) ? (w >> 16) : (w & 0xffffu);
    };
    // loader lane lq of 256 owns the elements k = 0..7 at row 16 I + 2 k + lq / 128, column 16 (I - 7) + lq mod 128
    // (consecutive lanes, consecutive columns: conflict-free window writes)
    const int lq = 64 * band_loader_slot(wv) + lane, lrow = lq >> 7, lcol = lq & 127;
    int lbk[8];
    uint32_t lok = 0;   // bit k: element k is a stored entry (kept apart from lbk: overwriting a register with a
                        // load in flight waits for the load, which put the block-index latency on the step)
    double lval[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { lbk[k] = -1; lval[k] = 0.0; }
    lds_barrier();
    CSTAMP(4);

    const BandSys SY{A, y, Lg};
    if (wv == 0) factor_block8(SY, Nl[0], NDl[0], 0, lane);
    lds_barrier();
    CSTAMP(5);
#ifdef LH_STAMPS
    unsigned long long ss_[5] = {0, 0, 0, 0, 0}, sa_ = __builtin_amdgcn_s_memtime(), sb_, bst_ = sa_;
    uint32_t su_ = 0;
#endif
    for (int t = 0; t < nstep; ++t) {
        const int k0 = 8 * t, par = t & 1, m0 = k0 + 8;
        const double* N = Nl[par];
        const double* ND = NDl[par];
        if (wv == BZW) {
            if (lane < 8) {   // z_t = b_t N_t, zeroed where |D| <= DBL_MIN (LDLT::_solve_impl)
                double zz = 0.0;
#pragma unroll
                for (int q = 0; q < 8; ++q) zz += y[k0 + q] * N[q * 8 + lane];
                const double d = SY.at(k0 + lane, k0 + lane);
                z[k0 + lane] = fabs(d) > 2.2250738585072014e-308 ? zz : 0.0;
            }
            NDg[64 * t + lane] = ND[lane];   // the back substitution's copy, off wave 0's chain
        }
        if (m0 < nb) {
            const int g0 = m0 >> 4;
            const uint32_t uw = unit_word(t);
#ifdef LH_STAMPS
            su_ = uw;
#endif
            if (wv == 0) {
                if (uw & LH_UNIT_VALID) {
                    diag_tile(SY, N, ND, k0, 16 * g0, lane);
                    wave_sync();
                }
                LDLT_SSTAMP(0);
                factor_block8(SY, Nl[par ^ 1], NDl[par ^ 1], m0, lane);
                LDLT_SSTAMP(1);
            } else if ((LU || !band_loader(wv)) && (uw & LH_UNIT_VALID)) {   // LU: the loaders too (steps of 12-15 units)
                const int I = g0 + (uw & 7), jb0 = g0 + ((uw >> 3) & 7), jb1 = g0 + ((uw >> 6) & 15);
                ldlt_tile_row(SY, N, ND, k0, 16 * I, 16 * jb0, 16 * jb1, -1, (uw & LH_UNIT_STORE) != 0, lane);
            }
            if (wv != 0) LDLT_SSTAMP(3);
        }
        if (band_loader(wv)) {
            // tile row I enters the window at step 2 I - 14, into the slots of tile row I - 8 (retired
            // after step 2 I - 15).  From the band image (prm.bimg, one rank) its values are loaded at step
            // 2 I - 16, in pairs; from the packed blocks (sharded solves) its block indices at 2 I - 16 and its
            // values at 2 I - 15
            // Every load is unconditional (clamped index): a conditional load becomes a branch whose join
            // waits for it.  Selections and the diagonal's lambda wait until the values are written.
            if ((t & 1) == 0) {
                const int Iw = t / 2 + 7;
                if (Iw >= 8 && Iw < NT) {
#ifdef LH_STAMPS
                    // (diagnostic) loader wave 12: the wait for its value loads, then the window writes
                    unsigned long long lt0_ = __builtin_amdgcn_s_memtime();
                    __builtin_amdgcn_s_waitcnt(0);
                    __builtin_amdgcn_sched_barrier(0);
                    unsigned long long lt1_ = __builtin_amdgcn_s_memtime();
                    if (wv == 12 && lane == 0) atomicAdd(&lh_stamps[56], lt1_ - lt0_);
#endif
                    if (bim) {
                        // pairs: lane lq holds columns 2 (lq mod 64) + {0, 1} of rows 16 Iw + 4 k + lq / 64 (lval[2k],
                        // lval[2k + 1]): one 16-byte store each, consecutive lanes on consecutive pairs
                        const int c = 16 * (Iw - 7) + 2 * (lq & 63);
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const int r = 16 * Iw + 4 * k + (lq >> 6);
                            double v0 = lval[2 * k], v1 = lval[2 * k + 1];
                            if (r == c) v0 = (r >= n) ? 1.0 : ((prm.strategy == 0) ? v0 + lambda : v0 + lambda * v0);
                            if (r == c + 1) v1 = (r >= n) ? 1.0 : ((prm.strategy == 0) ? v1 + lambda : v1 + lambda * v1);
                            *reinterpret_cast<double2*>(&SY.at(r, c)) = double2{(c <= r) ? v0 : 0.0, (c + 1 <= r) ? v1 : 0.0};
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < 8; ++k) {
                            const int r = 16 * Iw + 2 * k + lrow, c = 16 * (Iw - 7) + lcol;
                            double v = ((lok >> k) & 1) ? lval[k] : 0.0;
                            if (r == c) v = (r >= n) ? 1.0 : ((prm.strategy == 0) ? v + lambda : v + lambda * v);
                            SY.at(r, c) = (c <= r) ? v : 0.0;
                        }
                    }
#ifdef LH_STAMPS
                    __builtin_amdgcn_s_waitcnt(0);
                    __builtin_amdgcn_sched_barrier(0);
                    if (wv == 12 && lane == 0) {
                        atomicAdd(&lh_stamps[57], __builtin_amdgcn_s_memtime() - lt1_);
                        atomicAdd(&lh_stamps[58], 1ull);
                    }
#endif
                }
                const int Ia = t / 2 + 8;
                if (bim && Ia < NT) {
                    // tile row Ia's values from the band image, two steps before they are written: the pair at
                    // row 16 Ia + 4 k + lq / 64, columns 16 (Ia - 7) + 2 (lq mod 64) + {0, 1} is double2 256 k + lq
                    const double2* __restrict__ bt = reinterpret_cast<const double2*>(bsrc + (size_t)Ia * LH_BIMG_TR) + lq;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const double2 v = bt[256 * k];
                        lval[2 * k] = v.x;
                        lval[2 * k + 1] = v.y;
                    }
                } else if (Ia < NT) {
                    const int c = 16 * (Ia - 7) + lcol, pc = c / 6;
                    lok = 0;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const int r = 16 * Ia + 2 * k + lrow, pr = r / 6, d = pr - pc;
                        lbk[k] = bblk[min(max(pc, 0), P - 1) * 64 + min(max(d, 0), 63)];
                        lok |= (c <= r && r < n && d < 64) ? (1u << k) : 0u;
                    }
                }
            } else if (!bim) {
                const int Ib = (t - 1) / 2 + 8;
                if (Ib < NT) {
                    const int c = 16 * (Ib - 7) + lcol;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const int r = 16 * Ib + 2 * k + lrow;
                        lval[k] = src[(size_t)max(lbk[k], 0) * 36 + (c % 6) * 6 + (r % 6)];
                        if (lbk[k] < 0) lok &= ~(1u << k);   // a pair no chunk couples
                    }
                }
            }
        }
#ifdef LH_STAMPS
        // (diagnostic) each wave's arrival at the step barrier, from its own exit of the previous one
        if (lane == 0) atomicAdd(&lh_stamps[128 + 16 * (t & 1) + wv], __builtin_amdgcn_s_memtime() - bst_);
#endif
        lds_barrier();
#ifdef LH_STAMPS
        bst_ = __builtin_amdgcn_s_memtime();
#endif
        if (wv == 0) LDLT_SSTAMP(2); else LDLT_SSTAMP(4);
    }
#ifdef LH_STAMPS
    if (lane == 0) {
        if (wv == 0) {
            atomicAdd(&lh_stamps[46], ss_[0]);
            atomicAdd(&lh_stamps[47], ss_[1]);
            atomicAdd(&lh_stamps[48], ss_[2]);
            atomicAdd(&lh_stamps[51], 1ull);
        } else {
            atomicAdd(&lh_stamps[49], ss_[3]);
            atomicAdd(&lh_stamps[50], ss_[4]);
        }
    }
#endif
    __syncthreads();   // L and ND rows in global memory, z in LDS
    CSTAMP(6);

    // ---------------- back substitution x = L^-T z, blocks descending, one wave ----------------
    // The rows a block updates (L[KB+v][r] != 0 needs r >= KB + v - 104) live in registers: lane l,
    // slot s holds the row r = l + 64 s (mod 128) of the window [KB - 120, KB + 8), so the block's own 8
    // rows sit in 8 consecutive lanes of one 16-lane row (DPP broadcasts, as k_ctrl's backsub_block),
    // and once solved their lanes take the rows 128 below, which enter the window for the next block.
    // Per block: x_b = ND_b y_b, then every other held row takes y_r -= sum_v L[KB+v][r] x_b[v]; the
    // next block's L rows and ND are loaded while this one computes.
    // The L rows and ND come from global memory through an LDS ring the other 15 waves fill ahead of
    // wave 0 (the window's LDS is free now): block j of the descent (KB = nb - 8 - 8 j) goes to slot
    // j mod BRING, loaded by wave 1 + j mod 15 once wave 0 has read block j - BRING, and published by
    // a workgroup-scope release of bring_ready[slot] = j + 1.  Wave 0 reads each block's L from LDS one
    // block ahead (its ND when it starts the block).
    constexpr int BSLOT = 8 * LH_LBW + 64;   // one block: its 8 L rows as stored, then its ND
    constexpr int BRING = (128 * AS) / BSLOT;
    static_assert(BRING >= 15, "ring deeper than the producer count");
    __shared__ int bring_ready[BRING], bring_used;
    const int nblk = nb / 8;
    if (tid < BRING) bring_ready[tid] = 0;
    if (tid == 0) bring_used = 0;
    lds_barrier();
    if (wv > 0) {   // producers
        for (int j = wv - 1; j < nblk; j += 15) {
            if (j >= BRING)
                while (__hip_atomic_load(&bring_used, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < j - BRING + 1)
                    __builtin_amdgcn_s_sleep(1);
            const int KB = nb - 8 - 8 * j;
            const double2* gl = reinterpret_cast<const double2*>(Lg + (size_t)KB * LH_LBW);
            const double2* gn = reinterpret_cast<const double2*>(NDg + (size_t)8 * KB);
            double2 v[8], vn = double2{0.0, 0.0};
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = gl[k * 64 + lane];
            if (lane < 32) vn = gn[lane];
            double2* dst = reinterpret_cast<double2*>(A + (j % BRING) * BSLOT);
#pragma unroll
            for (int k = 0; k < 8; ++k) dst[k * 64 + lane] = v[k];
            if (lane < 32) dst[8 * 64 + lane] = vn;
            __hip_atomic_store(&bring_ready[j % BRING], j + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    } else {
      // NW (band_narrow: every row's envelope within 56 rows of its block): one held row per lane, the
      // window [KB - 56, KB + 8); else two, the window [KB - 120, KB + 8)
      auto consumer = [&](auto nw_tag) {
        constexpr bool NW = decltype(nw_tag)::value;
        constexpr int WROWS = NW ? 64 : 128;
        auto row_of = [&](int KB, int sl) {
            const int lo = KB + 8 - WROWS;
            return lo + ((lane + 64 * sl - lo) & (WROWS - 1));
        };
        // every block in [j0, j1] published (one round trip for the batch; producers run far ahead)
        auto wait_ready = [&](int j0, int j1) {
            for (;;) {
                int miss = 0;   // every flag read in one round trip (no short circuit)
                for (int j = j0; j <= j1; ++j)
                    miss |= __hip_atomic_load(&bring_ready[j % BRING], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != j + 1;
                if (!miss) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   // orders the slot reads after
                    return;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        };
        // block j's L entries of this lane's two rows from its slot (clamped: the own block's rows and rows
        // past the band read in-bounds values never used)
        // (a held row is >= KB - 120 >= KB + v - LH_LBW, inside every stored L row: one clamp, and the 8 reads
        // of a row share one address, v (LH_LBW - 1) doubles apart as immediate offsets)
        auto load_blk = [&](int j, double (&l0)[8], double (&l1)[8]) {
            const int KB = nb - 8 - 8 * j;
            const double* sl = A + (j % BRING) * BSLOT + LH_LBW - KB;   // + v (LH_LBW - 1) + r: L[KB+v][r]
            const double* p0 = sl + min(row_of(KB, 0), KB - 1);
            const double* p1 = sl + min(row_of(KB, 1), KB - 1);
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                l0[v] = p0[v * (LH_LBW - 1)];
                l1[v] = NW ? 0.0 : p1[v * (LH_LBW - 1)];
            }
        };
        double y0, y1;
        {
            const int r0 = row_of(nb - 8, 0), r1 = row_of(nb - 8, 1);
            y0 = (r0 >= 0) ? z[r0] : 0.0;
            y1 = (!NW && r1 >= 0) ? z[r1] : 0.0;
        }
        // block j with its L entries ca / cb: x_b = ND_b y_b, then the held rows' updates
#ifdef LH_STAMPS
        unsigned long long bs_[3] = {0, 0, 0}, ba_ = 0, bb_ = 0;
#define BSUB_STAMP(i) do { __builtin_amdgcn_sched_barrier(0); bb_ = __builtin_amdgcn_s_memtime(); \
        if ((i) >= 0) bs_[(i) < 0 ? 0 : (i)] += bb_ - ba_; ba_ = bb_; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define BSUB_STAMP(i)
#endif
        // block j's ND row (lane & 7) from its slot
        auto load_nd = [&](int j, double (&cn)[8]) {
            const double* p = A + (j % BRING) * BSLOT + 8 * LH_LBW + (lane & 7) * 8;
#pragma unroll
            for (int v = 0; v < 8; ++v) cn[v] = p[v];
        };
        double cn[8];   // block j's ND row on entry; block j + 1's, loaded once x_b is formed, on exit
        auto solve_blk = [&](int j, const double (&ca)[8], const double (&cb)[8]) {
            BSUB_STAMP(-1);
            const int KB = nb - 8 - 8 * j;
            const int sb_ = NW ? 0 : (KB >> 6) & 1, kl = KB & 63;
            const bool mine = lane >= kl && lane < kl + 8;
            const int re = KB - WROWS + (lane - kl);                     // the row entering this lane's slot
            const double zin = z[max(re, 0)];
            const double ys = sb_ ? y1 : y0;
            double yb[8];
            if (KB & 8) {
                yb[0] = bcast16<8>(ys); yb[1] = bcast16<9>(ys); yb[2] = bcast16<10>(ys); yb[3] = bcast16<11>(ys);
                yb[4] = bcast16<12>(ys); yb[5] = bcast16<13>(ys); yb[6] = bcast16<14>(ys); yb[7] = bcast16<15>(ys);
            } else {
                yb[0] = bcast16<0>(ys); yb[1] = bcast16<1>(ys); yb[2] = bcast16<2>(ys); yb[3] = bcast16<3>(ys);
                yb[4] = bcast16<4>(ys); yb[5] = bcast16<5>(ys); yb[6] = bcast16<6>(ys); yb[7] = bcast16<7>(ys);
            }
            const double xv = ((cn[0] * yb[0] + cn[1] * yb[1]) + (cn[2] * yb[2] + cn[3] * yb[3])) +
                              ((cn[4] * yb[4] + cn[5] * yb[5]) + (cn[6] * yb[6] + cn[7] * yb[7]));
            load_nd(min(j + 1, nblk - 1), cn);   // published: j + 1 < j + 4, checked an iteration before
#ifdef LH_STAMPS
            double xvs = xv;
            asm volatile("" : "+v"(xvs));
#endif
            BSUB_STAMP(0);
            double xb[8];
#pragma unroll
            for (int v = 0; v < 8; ++v) xb[v] = readlane_d(xv, kl + v);
            const double sa = ((ca[0] * xb[0] + ca[1] * xb[1]) + (ca[2] * xb[2] + ca[3] * xb[3])) +
                              ((ca[4] * xb[4] + ca[5] * xb[5]) + (ca[6] * xb[6] + ca[7] * xb[7]));
            // rows past the band have zero L; the block's own rows (r >= KB) take no update
            if (row_of(KB, 0) < KB) y0 -= sa;
            if constexpr (!NW) {
                const double sbb = ((cb[0] * xb[0] + cb[1] * xb[1]) + (cb[2] * xb[2] + cb[3] * xb[3])) +
                                   ((cb[4] * xb[4] + cb[5] * xb[5]) + (cb[6] * xb[6] + cb[7] * xb[7]));
                if (row_of(KB, 1) < KB) y1 -= sbb;
            }
            if (mine) {
                y[KB + (lane - kl)] = xv;                                // the solution, natural order
                const double zi = re >= 0 ? zin : 0.0;
                if (sb_) y1 = zi; else y0 = zi;
            }
#ifdef LH_STAMPS
            asm volatile("" : "+v"(y0), "+v"(y1));
#endif
            BSUB_STAMP(1);
        };
        // two register sets in turn (no copies between blocks); every 4 blocks one batched readiness check
        // for the next 4 and one release of the slots read so far (the release waits for this wave's
        // outstanding LDS reads, so no producer rewrites a slot still being read)
        double la[8], lb[8], ma[8], mb[8];
        wait_ready(0, min(3, nblk - 1));
        load_blk(0, la, lb);
        load_nd(0, cn);
        for (int j = 0; j < nblk; j += 2) {
            // the flags of blocks j + 4 .. j + 7 (first loaded at iteration j + 2) are read now and checked
            // after block j, so the read's round trip overlaps the block instead of preceding it
            const bool chk = (j & 3) == 0 && j + 4 < nblk;
            int miss = 0;
            if (chk)
                for (int q = j + 4; q <= min(j + 7, nblk - 1); ++q)
                    miss |= __hip_atomic_load(&bring_ready[q % BRING], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != q + 1;
            load_blk(min(j + 1, nblk - 1), ma, mb);
            solve_blk(j, la, lb);
            BSUB_STAMP(-1);
            if (chk) {
                if (miss) wait_ready(j + 4, min(j + 7, nblk - 1));
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
            BSUB_STAMP(2);
            if (j + 1 >= nblk) break;
            load_blk(min(j + 2, nblk - 1), la, lb);
            solve_blk(j + 1, ma, mb);
            if ((j & 3) == 2 && lane == 0)
                __hip_atomic_store(&bring_used, j + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
#ifdef LH_STAMPS
        if (lane == 0) {
            atomicAdd(&lh_stamps[52], bs_[0]);
            atomicAdd(&lh_stamps[53], bs_[1]);
            atomicAdd(&lh_stamps[54], bs_[2]);
            atomicAdd(&lh_stamps[55], (unsigned long long)nblk);
        }
#endif
#undef BSUB_STAMP
      };
      if (prm.band_narrow) consumer(BoolTag<true>{});
      else consumer(BoolTag<false>{});
    }
    __syncthreads();
    CSTAMP(8);
    ctrl_step_tail<CT>(ctrl, prm, n, lambda, y, src + LY.off_bp, src + LY.off_hd, s_red, dxp, rung);
    CSTAMP(12);
#ifdef LH_STAMPS
    if (tid == 0) atomicAdd(&lh_stamps[63], (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
}

// ============================================================================
// k_ctrl_p: the controller with the reduced pose system solved by PCG (lh_options.linear_solver =
// PCG) past LH_PMAX poses, up to LH_PMAX_ANY (windows of many keyframes).  One
// 1024-thread workgroup.  Same LM bookkeeping (ctrl_lm_step) and step tail (ctrl_step_tail) as the
// other controllers.  S stays in the packed blocks k_reduce wrote (rs: one 6x6 block per pose pair
// that some landmark couples, plus every diagonal block; lh_plan.cpp), never densified: the PCG's
// S p walks each pose's block row (Plan::brow_ent, ascending column) straight from the packed
// blocks, 6 rows per pose, one thread per row.  The algorithm is the reference's Problem::PCGSolver
// (problem.cpp:584-614) with its first-step bug fixed, as the oracle's pcg_solve restates it: Jacobi
// preconditioner on S + lambda D, stop when ||r|| <= pcg_tol ||b|| (1e-6, :597), at most 2 n steps
// after the first (:422); a zero diagonal preconditions with 0.  The dot products are fixed-order
// workgroup reductions (wave butterflies, then the 16 wave sums in order), so a solve is bitwise
// repeatable; the sums' order differs from the oracle's sequential loops (parity to tolerance).
// ============================================================================
#define PNMAX (6 * LH_PMAX_ANY)
#define PRT ((PNMAX + CT - 1) / CT)     // rows per thread

// fixed-order workgroup sum of one value per thread (every thread gets the total); red: 16 doubles
__device__ __forceinline__ double wg_sum(double v, double* red, int lane, int wave) {
    double g[1] = {v};
    group_sum(g, 6);   // DPP and permlane butterflies, lane ^ 1 .. ^ 32
    v = g[0];
    if (lane == 0) red[wave] = v;
    lds_barrier();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < CT / 64; ++w) t += red[w];
    return t;
}

__global__ __launch_bounds__(CT) void k_ctrl_p(lh_ctrl* __restrict__ ctrl, double* __restrict__ rs_commit,
                                               const double* __restrict__ rs_stage, const double* __restrict__ maxd_in,
                                               const int32_t* __restrict__ brow_ptr, const uint32_t* __restrict__ brow_ent,
                                               double* __restrict__ dxp, lh_params prm,
                                               int mode, volatile int* __restrict__ host_done, int seq,
                                               double* __restrict__ ell) {
    __shared__ double pv[PNMAX], bpv[PNMAX], hdv[PNMAX], xs[PNMAX];
    __shared__ int s_flags[4];
    __shared__ __attribute__((aligned(16))) double s_red[3][CT / 64];
    __shared__ double s_lam;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int P = prm.P, n = 6 * P;
    const lh_rs_layout LY = lh_rs_make(P, prm.npairs);

    // ---------------- controller words, pose matrices, max |diag| (mode 0), the LM decision ----------------
    // workgroup `rung` > 0: a lambda-ladder rung with its own row copy of S; it waits for workgroup
    // 0's decision
    const int rung = (int)blockIdx.x;
#ifdef LH_STAMPS
    if (rung) return;
#endif
    if (rung && mode == 0) return;   // (the initial linearisation builds no ladder, as k_ctrl)
    if (rung) {
        ladder_wait(ctrl, seq);
        const LadderDec d = ladder_read(ctrl, prm, seq, rung);
        if (tid == 0) {
            s_flags[0] = d.done;
            s_flags[1] = d.accept;
            s_flags[3] = d.skip;
            s_lam = d.lambda;
        }
        lds_barrier();
    }
    double tchi = 0.0, sl = 0.0, ndg = 0.0;
    CtrlWords cw{};
    if (tid == 0 && !rung) {
        cw = ctrl_load(ctrl);
        tchi = 0.5 * rs_stage[LY.off_sc + LH_SC_CHI2];
        sl = rs_stage[LY.off_sc + LH_SC_SCALE];
        ndg = rs_stage[LY.off_sc + LH_SC_NDEG];
    }
    if (!rung) {
        double mx = 0.0;
        if (mode == 0)
            for (int i = tid; i < n; i += CT) mx = fmax(mx, fabs(rs_stage[LY.off_hd + i]));
        for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
        if (lane == 0) s_red[0][wave] = mx;
    }
    lds_barrier();
    if (tid == 0 && !rung) {
        double mdiag = 0.0;
        if (mode == 0) {
            for (int w = 0; w < CT / 64; ++w) mdiag = fmax(mdiag, s_red[0][w]);
            mdiag = fmax(*maxd_in, mdiag);
        }
        int done, accept, cur;
        double lam_n;
        __shared__ int b_cnt[4];
        s_flags[3] = ctrl_decide(ctrl, cw, prm, mode, mdiag, tchi, sl, ndg, rs_stage, LY, host_done, seq, done, accept, cur,
                                 lam_n, b_cnt);
        if (prm.ladder > 1 && mode != 0) ladder_publish(ctrl, seq);   // the rung workgroups wait for it
        s_flags[0] = done;
        s_flags[1] = accept;
        s_flags[2] = cur;
        s_lam = lam_n;
    }
    lds_barrier();
    const int done = s_flags[0], accept = s_flags[1];
    if (done || s_flags[3]) return;   // stopped, an evaluate-only acceptance, or a rejection onto a built rung
    const double lambda = s_lam;
    {
        const bool build = mode != 0 && ladder_build(prm, accept);
        if (rung != 0 && (!build || rung >= prm.ladder)) return;
        if (rung == 0 && tid == 0) ctrl->lad_n = build ? prm.ladder : 1;
        ell += (size_t)rung * prm.lad_stride;
        dxp += (size_t)rung * n;
    }

    // ---------------- the chosen system (the candidate's on accept, committed on it; else the committed one) ----------------
    const double* __restrict__ src = accept ? rs_stage : rs_commit;
    if (accept && rung == 0)
        for (int i = tid; i < LY.total; i += CT) rs_commit[i] = rs_stage[i];
    const double* __restrict__ Sb = src + LY.off_S;
    // per thread rows r = tid + CT u: damped diagonal, Jacobi preconditioner, right-hand side
    double dr[PRT], minv[PRT], x[PRT], rr[PRT], z[PRT], pp[PRT];
    int e0[PRT], e1[PRT];
#pragma unroll
    for (int u = 0; u < PRT; ++u) {
        const int r = tid + CT * u;
        const bool in = r < n;
        const int p = in ? r / 6 : 0, a = r - 6 * p;
        e0[u] = in ? brow_ptr[p] : 0;
        e1[u] = in ? brow_ptr[p + 1] : 0;
        double sd = 0.0;
        for (int e = e0[u]; e < e1[u]; ++e) {   // the diagonal block: the entry whose column is p itself
            const uint32_t en = brow_ent[e];
            if ((int)((en >> 1) & 0xFFF) == p && !(en & 1u)) sd = Sb[(size_t)(en >> 13) * 36 + 7 * a];
        }
        dr[u] = (prm.strategy == 0) ? sd + lambda : sd + lambda * sd;   // problem.cpp:408-418
        minv[u] = (in && dr[u] != 0.0) ? 1.0 / dr[u] : 0.0;
        rr[u] = in ? src[LY.off_bs + r] : 0.0;
        x[u] = 0.0;
        z[u] = minv[u] * rr[u];
        pp[u] = z[u];
        if (in) { bpv[r] = src[LY.off_bp + r]; hdv[r] = src[LY.off_hd + r]; }
    }
    // Each row's entries gathered once per solve into row-contiguous scratch: entry e of pose p's block
    // row holds S(6p + a, 6q + c) at ell[(6 e + a) * 6 + c], the damped diagonal in place.  A step's
    // S p then reads 48 contiguous bytes per entry, at addresses that need no index word first (the
    // walk over the packed blocks put two dependent L2 round trips per entry on the chain).
#pragma unroll
    for (int u = 0; u < PRT; ++u) {
        const int r = tid + CT * u;
        if (r >= n) continue;
        const int p = r / 6, a = r - 6 * p;
        for (int e = e0[u]; e < e1[u]; ++e) {
            const uint32_t en = brow_ent[e];
            const int q = (int)((en >> 1) & 0xFFF);
            const double* blk = Sb + (size_t)(en >> 13) * 36;
            double* dst = ell + ((size_t)6 * e + a) * 6;
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                double val = (en & 1u) ? blk[6 * c + a] : blk[6 * a + c];   // (q, p) read transposed
                if (!(en & 1u) && q == p && c == a) val = dr[u];              // the damped diagonal
                dst[c] = val;
            }
        }
    }
    __syncthreads();   // the scratch is read back by the same threads: global stores visible to the loads below
    // Two barriers per step: z is published in pv and one product serves the step, q = (S + lambda D) z +
    // beta q_prev and p = z + beta p_prev (the same recurrence regrouped, as k_ctrl's PCG).  The dot
    // products are fixed-order sums (wave butterflies, then the 16 wave partials in order).
    double2* red2 = reinterpret_cast<double2*>(&s_red[1][0]);   // [16] (r.z, r.r) partials (s_red[1..2])
    double* red_pq = s_red[0];
    auto total2 = [&](double& tz, double& tr) {
        tz = 0.0;
        tr = 0.0;
#pragma unroll
        for (int w = 0; w < CT / 64; ++w) {
            const double2 t = red2[w];
            tz += t.x;
            tr += t.y;
        }
    };
    {
        double t2[2] = {0.0, 0.0};
#pragma unroll
        for (int u = 0; u < PRT; ++u) {
            t2[0] += rr[u] * z[u];
            t2[1] += rr[u] * rr[u];
            pp[u] = 0.0;
            if (tid + CT * u < n) pv[tid + CT * u] = z[u];
        }
        group_sum(t2, 6);
        if (lane == 0) red2[wave] = double2{t2[0], t2[1]};
    }
    lds_barrier();
    double rz, bb;
    total2(rz, bb);
    const double thr = prm.pcg_tol * sqrt(bb);
    const int maxit = prm.pcg_max_it > 0 ? prm.pcg_max_it : 2 * n;
    int steps = 0;
    double w[PRT], beta = 0.0;
#pragma unroll
    for (int u = 0; u < PRT; ++u) w[u] = 0.0;
    if (bb > 0.0) {
        for (;;) {
            // s = (S + lambda D) z, row by row over the block row, columns ascending
            double pw[1] = {0.0};
#pragma unroll
            for (int u = 0; u < PRT; ++u) {
                const int r = tid + CT * u;
                const int a = r - 6 * (r / 6);
                double acc = 0.0;
#pragma unroll 2
                for (int e = e0[u]; e < e1[u]; ++e) {
                    const int q = (int)((brow_ent[e] >> 1) & 0xFFF);
                    const double2* row = reinterpret_cast<const double2*>(ell + ((size_t)6 * e + a) * 6);
                    const double2 v0 = row[0], v1 = row[1], v2 = row[2];
                    const double* pq = pv + 6 * q;
                    acc += v0.x * pq[0];
                    acc += v0.y * pq[1];
                    acc += v1.x * pq[2];
                    acc += v1.y * pq[3];
                    acc += v2.x * pq[4];
                    acc += v2.y * pq[5];
                }
                w[u] = acc + beta * w[u];
                pp[u] = z[u] + beta * pp[u];
                pw[0] += pp[u] * w[u];
            }
            group_sum(pw, 6);
            if (lane == 0) red_pq[wave] = pw[0];
            lds_barrier();
            double tpw = 0.0;
#pragma unroll
            for (int wv = 0; wv < CT / 64; ++wv) tpw += red_pq[wv];
            const double alpha = rz / tpw;
            double a2[2] = {0.0, 0.0};
#pragma unroll
            for (int u = 0; u < PRT; ++u) {
                x[u] += alpha * pp[u];
                rr[u] -= alpha * w[u];
                z[u] = minv[u] * rr[u];
                a2[0] += rr[u] * z[u];
                a2[1] += rr[u] * rr[u];
                if (tid + CT * u < n) pv[tid + CT * u] = z[u];
            }
            group_sum(a2, 6);
            if (lane == 0) red2[wave] = double2{a2[0], a2[1]};
            lds_barrier();
            double rzn, rrn;
            total2(rzn, rrn);
            ++steps;
            if (!(sqrt(rrn) > thr) || steps >= maxit + 1) break;   // also stops on NaN
            beta = rzn / rz;
            rz = rzn;
        }
    }
#pragma unroll
    for (int u = 0; u < PRT; ++u) {
        const int r = tid + CT * u;
        if (r < n) { xs[r] = x[u]; dxp[r] = x[u]; }
    }
    if (tid == 0) {
        ctrl->lad_its[rung] = steps;
        if (rung == 0) ctrl->pcg_iters += steps;   // a higher rung's count is added when a rejection uses it
    }
    lds_barrier();
    ctrl_step_tail<CT>(ctrl, prm, n, lambda, xs, bpv, hdv, s_red[0], nullptr, rung);
}

// ============================================================================
// k_frames: the frontend's pose-only LM, Frontend::EstimateCurrentPose
// (src/frontend_lego.cpp:157-250), one workgroup per frame, the whole thing in
// one launch: four rounds of problem.solve(10) on one VertexPose with
// EdgeProjectionPoseOnly edges (lego_types.h:116-180), each round restarting
// from the frame's pose, then the outlier flags (:205-226); the edges lose the
// Huber cost after round three (:223-225).  Edges are never removed (the
// reference's setLevel is commented out).  n = 6: the Schur complement is H_pp
// itself (problem.cpp:380-430 with no landmark vertex), solved by wave 0 in
// registers with Eigen's pivoted LDLT (po_ldlt6_wave).  Per-edge arithmetic is the bitwise mirror of
// oracle/lego_oracle.c (po_residual / po_jacobian); sums have a fixed order
// (thread-strided, then a fixed tree), so a batch is bitwise reproducible.
// ============================================================================
#define FT 256                 // threads per frame
#define FV 28                  // per-edge sums: H_pp upper (21) | b (6) | rho0
#pragma clang fp contract(off)

// EdgeProjectionPoseOnly residual + Jacobian at pos_cam = T X (one transform for both)
__device__ __forceinline__ void po_edge(const double* q, const double* t, const double X[3], double u, double v,
                                        const double* K, double& r0, double& r1, double J[12], bool want_j) {
    double Pc[3];
    d_q_rotate(q, X, Pc);
#pragma unroll
    for (int i = 0; i < 3; ++i) Pc[i] = Pc[i] + t[i];
    double p0 = K[0] * Pc[0] + K[2] * Pc[2];
    double p1 = K[1] * Pc[1] + K[3] * Pc[2];
    const double den = Pc[2] + 1e-18;
    p0 /= den;
    p1 /= den;
    r0 = u - p0;
    r1 = v - p1;
    if (want_j) {
        const double fx = K[0], fy = K[1];
        const double x = Pc[0], y = Pc[1], z = Pc[2];
        const double zi = 1.0 / (z + 1e-18);
        const double zi2 = zi * zi;
        J[0] = -fx * zi;              J[1] = 0.0;                  J[2] = fx * x * zi2;
        J[3] = fx * x * y * zi2;      J[4] = -fx - fx * x * x * zi2; J[5] = fx * y * zi;
        J[6] = 0.0;                   J[7] = -fy * zi;             J[8] = fy * y * zi2;
        J[9] = fy + fy * y * y * zi2; J[10] = -fy * x * y * zi2;   J[11] = -fy * x * zi;
    }
}

__device__ __forceinline__ double po_rho0(double r0, double r1, double delta) {
    const double e2 = r0 * r0 + r1 * r1;
    if (delta > 0.0) {
        const double d2 = delta * delta;
        if (e2 <= d2) return e2;
        const double s = sqrt(e2);
        return 2 * s * delta - d2;
    }
    return e2;
}

// one edge's contributions: (J^T W) J upper triangle, -(rho1 J)^T r, rho0  (problem.cpp:300-330).
// The products contract to FMAs: these sums are parity-to-tolerance (their order differs from the oracle's
// anyway); edge_robust keeps the bitwise-mirrored gate (contraction is fixed where an expression is written).
#pragma clang fp contract(fast)
__device__ __forceinline__ void po_accumulate(double r0, double r1, const double J[12], double delta, double acc[FV]) {
    EdgeEval E;
    E.r0 = r0; E.r1 = r1;
    lh_params pr{};
    pr.huber_delta = delta;
    edge_robust(E, pr);
    double JtW[12];
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        JtW[2 * a] = J[a] * E.W00 + J[6 + a] * E.W10;
        JtW[2 * a + 1] = J[a] * E.W01 + J[6 + a] * E.W11;
    }
    int k = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int c = a; c < 6; ++c) acc[k++] += JtW[2 * a] * J[c] + JtW[2 * a + 1] * J[6 + c];
#pragma unroll
    for (int a = 0; a < 6; ++a) acc[21 + a] -= (E.rho1 * J[a]) * r0 + (E.rho1 * J[6 + a]) * r1;
    acc[27] += E.rho0;
}
#pragma clang fp contract(off)

// The oracle's ldlt_solve (Eigen ldlt_inplace with diagonal pivoting + LDLT::_solve_impl) for n = 6,
// in registers: every lane holds the whole symmetric system and runs the oracle's operations in the
// oracle's order, so no value crosses lanes.  Two changes: multiply-adds contract to FMAs, and a division
// by a pivot is its reciprocal (fast_rcp, one per pivot) times the element, as the k_ctrl LDL^T does.  The
// frontend's sums of H and b already differ from the oracle's order, so its parity is to tolerance
// either way (tests/test_frontend.py), and the 21 IEEE divisions were the longest part of the step.
// The damped system is read from LDS (H full symmetric, b), with Eigen's pivot sequence found first: Eigen's left-looking ldlt_inplace compares diagonal entries no earlier step has changed, so its
// transpositions depend on the damped diagonal alone.  They are replayed on six (key, row) pairs, the
// permuted system is loaded from LDS at the permuted addresses, the factorisation and the solves run
// without swaps (the same operations on the same values as Eigen's in-place swapping loop, so the same
// bits as a swapping version), and x goes back to pose order through LDS.  This keeps the 36-element row
// and column exchanges (a branch per candidate row per step) off the chain.
#pragma clang fp contract(fast)   // the 6x6 solve is parity-to-tolerance (see above): FMAs halve its chains
__device__ __forceinline__ void po_ldlt6_lds(const double* H, const double* bv, double lam, int strategy,
                                             double* xs, double (&x)[6]) {
    double key[6];
    int pos[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const double h = H[7 * i];
        key[i] = h + ((strategy == 0) ? lam : lam * h);
        pos[i] = i;
    }
    bool all_zero = false;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int idx = k;
        double big = fabs(key[k]);
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            const double di = fabs(key[i]);
            if (di > big) { big = di; idx = i; }
        }
        idx = __builtin_amdgcn_readfirstlane(idx);
        if (k == 0 && !(big > 0.0)) { all_zero = true; break; }   // Eigen: identity transpositions
#pragma unroll
        for (int m = k + 1; m < 6; ++m)
            if (m == idx) {
                const double t = key[k]; key[k] = key[m]; key[m] = t;
                const int u = pos[k]; pos[k] = pos[m]; pos[m] = u;
            }
    }
    double A[6][6], y[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
#pragma unroll
        for (int c = 0; c < 6; ++c) A[r][c] = H[6 * pos[r] + pos[c]];
        A[r][r] += (strategy == 0) ? lam : lam * A[r][r];
        y[r] = bv[pos[r]];
    }
    if (!all_zero) {
        double dd[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            if (k > 0) {
                double temp[6];
#pragma unroll
                for (int j = 0; j < k; ++j) temp[j] = dd[j] * A[k][j];
#pragma unroll
                for (int r = k; r < 6; ++r) {
                    double si = 0.0;
#pragma unroll
                    for (int j = 0; j < k; ++j) si += A[r][j] * temp[j];
                    A[r][k] -= si;
                }
            }
            const double akk = A[k][k];
            dd[k] = akk;
            if (k < 5 && fabs(akk) > 0.0) {
                const double inv = fast_rcp(akk);
#pragma unroll
                for (int r = k + 1; r < 6; ++r) A[r][k] *= inv;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 6; ++k)
        if (y[k] != 0.0)
#pragma unroll
            for (int i = k + 1; i < 6; ++i) y[i] -= A[i][k] * y[k];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const double d = A[i][i];
        y[i] = (fabs(d) > 2.2250738585072014e-308) ? y[i] * fast_rcp(d) : 0.0;
    }
#pragma unroll
    for (int k = 5; k >= 0; --k)
#pragma unroll
        for (int i = 0; i < k; ++i) y[i] -= A[k][i] * y[k];
#pragma unroll
    for (int r = 0; r < 6; ++r) xs[pos[r]] = y[r];   // every lane writes the same value
    wave_sync();
#pragma unroll
    for (int j = 0; j < 6; ++j) x[j] = xs[j];
}

#pragma clang fp contract(off)
// sin and cos of |x| <= 0.8 by their Taylor series to x^17 / x^18 in Horner form on x^2 (the next terms are
// below 1e-19): within 1 ulp of the host libm's sin / cos (2e7 samples, 1-2 % of them 1 ulp apart; the
// device library's sincos is not bitwise the host's either).  A frame's pose step is small, so its angle
// takes this path; larger ones take the library's sincos.
__device__ __forceinline__ void po_sincos_small(double x, double& s, double& c) {
    const double x2 = x * x;
    double p = -8.22063524662433e-18;
    p = __builtin_fma(p, x2, 2.8114572543455206e-15);
    p = __builtin_fma(p, x2, -7.647163731819816e-13);
    p = __builtin_fma(p, x2, 1.6059043836821613e-10);
    p = __builtin_fma(p, x2, -2.505210838544172e-08);
    p = __builtin_fma(p, x2, 2.7557319223985893e-06);
    p = __builtin_fma(p, x2, -0.0001984126984126984);
    p = __builtin_fma(p, x2, 0.008333333333333333);
    p = __builtin_fma(p, x2, -0.16666666666666666);
    s = __builtin_fma(x * x2, p, x);
    double q = 4.110317623312165e-19;
    q = __builtin_fma(q, x2, -1.5619206968586225e-16);
    q = __builtin_fma(q, x2, 4.779477332387385e-14);
    q = __builtin_fma(q, x2, -1.1470745597729725e-11);
    q = __builtin_fma(q, x2, 2.08767569878681e-09);
    q = __builtin_fma(q, x2, -2.755731922398589e-07);
    q = __builtin_fma(q, x2, 2.48015873015873e-05);
    q = __builtin_fma(q, x2, -0.001388888888888889);
    q = __builtin_fma(q, x2, 0.041666666666666664);
    q = __builtin_fma(q, x2, -0.5);
    c = __builtin_fma(x2, q, 1.0);
}
// the library's sincos out of line (its registers are not live across the frame's pose update)
__device__ __attribute__((noinline)) double2 po_sincos_libm(double x) {
    double s, c;
    sincos(x, &s, &c);
    return double2{s, c};
}
// VertexPose::add: T12 <- (SE3::exp(d) * SE3(T12)).matrix(), NaN/Inf step -> zero (lego_types.h:61-91),
// on one wave: every lane computes the same result, except that lane 0 takes sin/cos(theta/2) and
// lane 1 sin/cos(theta) in one sincos pass.  qT = the quaternion of SE3(T12) (d_q_from_R of its
// rotation), cached by the caller.  out12: the new pose matrix (every lane), q/t: its SE3 table.
__device__ __forceinline__ void po_pose_add_wave(const double (&d_in)[6], const double* T12, const double* qT,
                                                 double (&out12)[12], double (&qo)[4], double (&to)[3], int lane) {
    double d[6];
    bool bad = false;
#pragma unroll
    for (int a = 0; a < 6; ++a) { d[a] = d_in[a]; bad |= !isfinite(d[a]); }
    if (bad) {
#pragma unroll
        for (int a = 0; a < 6; ++a) d[a] = 0.0;
    }
    const double th = d_twist_theta(d);
    double sn, cs;
    const double ang = lane == 1 ? th : 0.5 * th;
#ifndef LH_PO_LIBM_SINCOS
    if (__builtin_amdgcn_readfirstlane((int)(th <= 0.8)))   // th: the same in every lane
        po_sincos_small(ang, sn, cs);
    else
    {
        const double2 r = po_sincos_libm(ang);
        sn = r.x;
        cs = r.y;
    }
#else
    sincos(ang, &sn, &cs);
#endif
    const double sh = readlane_d(sn, 0), ch = readlane_d(cs, 0), st = readlane_d(sn, 1), ct = readlane_d(cs, 1);
    double qe[4], te[3], qn[4], tr[3], Rn[9];
    d_se3_exp_trig(d, sh, ch, st, ct, qe, te);
    const double qTr[4] = {qT[0], qT[1], qT[2], qT[3]};
    const double tc[3] = {T12[3], T12[7], T12[11]};
    d_q_mul(qe, qTr, qn);
    d_q_rotate(qe, tc, tr);
    d_R_from_q(qn, Rn);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        out12[4 * i] = Rn[3 * i]; out12[4 * i + 1] = Rn[3 * i + 1]; out12[4 * i + 2] = Rn[3 * i + 2];
        out12[4 * i + 3] = te[i] + tr[i];
    }
    // SE3(estimate_) of the new matrix, as the next linearisation reads it
    const double R[9] = {out12[0], out12[1], out12[2], out12[4], out12[5], out12[6], out12[8], out12[9], out12[10]};
    d_q_from_R(R, qo);
    to[0] = out12[3]; to[1] = out12[7]; to[2] = out12[11];
}

#pragma clang fp contract(fast)

struct PoShared {
    double pose[12], cand[12], q[4], t[3], qp[4], K[4];   // q/t: the table being linearised; qp: SE3(pose)'s q
    double H[36], b[6], dx[6], xs[6];   // xs: the 6x6 solution on its way back to pose order
    double part[FT / 64][FV];
    double sum[FV];
    double rows[FT][FV + 1];   // one thread's per-edge sums per row (odd stride: column reads spread over banks)
    double chi, lam, ni, last, delta;
    int iter, fc, cont;        // completed iterations, rejected trials in the iteration, another trial follows
};

// all FT threads: each thread's acc[FV] through LDS rows; per wave, lane 2k + h (k < FV) sums column k
// over the wave's rows of parity h (four interleaved chains, fixed order), and the two halves are added: S.part[wave].
// The caller's barrier follows.  Fixed order: a batch is bitwise reproducible.
__device__ __forceinline__ void po_rows_to_parts(const double (&acc)[FV], PoShared& S, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int k = 0; k < FV; ++k) S.rows[tid][k] = acc[k];
    wave_sync();
    if (lane < 2 * FV) {
        const int k = lane >> 1, h = lane & 1;
        // four interleaved chains (rows i mod 4), then ((c0 + c1) + (c2 + c3)): a fixed order, a quarter of the
        // dependent adds
        double c[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int i = 0; i < 32; ++i) c[i & 3] += S.rows[64 * wave + 2 * i + h][k];
        double s = (c[0] + c[1]) + (c[2] + c[3]);
        s += dpp_d<0xB1>(s);   // quad_perm [1,0,3,2]: the other parity's half
        if (h == 0) S.part[wave][k] = s;
    }
}

// SE3(estimate_) of T12 into q / t (d_q_from_R of its rotation)
__device__ __forceinline__ void po_table_regs(const double* T12, double (&q)[4], double (&t)[3]) {
    const double R[9] = {T12[0], T12[1], T12[2], T12[4], T12[5], T12[6], T12[8], T12[9], T12[10]};
    d_q_from_R(R, q);
    t[0] = T12[3]; t[1] = T12[7]; t[2] = T12[11];
}

// One workgroup per frame.  Per LM trial there are two barriers: after the linearisation's per-wave
// sums, and after wave 0 has finished the sums, taken the LM decision (lane 0) and, when another
// trial follows, solved the 6x6 step and composed the candidate pose (all of wave 0).
__global__ __launch_bounds__(FT) void k_frames(const int64_t* __restrict__ obs_ptr, const double* __restrict__ pose_in,
                                               const double* __restrict__ pts, const double* __restrict__ uv,
                                               const uint8_t* __restrict__ flag_in, lh_params prm,
                                               double* __restrict__ res, double* __restrict__ pose_out,
                                               uint8_t* __restrict__ flag_out, double* __restrict__ rchi2_out,
                                               int32_t* __restrict__ iters_out, int32_t* __restrict__ inliers_out) {
    __shared__ PoShared S;
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t o0 = obs_ptr[f];
    const int O = (int)(obs_ptr[f + 1] - o0);
    const double* X = pts + 3 * o0;
    const double* Z = uv + 2 * o0;
    double* R = res + 2 * o0;
    uint8_t* flag = flag_out + o0;
    for (int e = tid; e < O; e += FT) flag[e] = flag_in ? (flag_in[o0 + e] != 0) : 0;
    if (tid < 4) S.K[tid] = prm.K[tid];
    if (tid == 0) S.delta = prm.huber_delta;
    int its = 0;
    STAMP_DECL   // diagnostic build: per-phase wave-cycles into lh_stamps[24..29]
    // this thread's first edge, in registers for the whole launch (a frame of <= FT edges then reads
    // no edge input from memory after this; further edges are read per pass)
    double X0[3] = {0.0, 0.0, 0.0}, Z0[2] = {0.0, 0.0};
    if (tid < O) {
        X0[0] = X[3 * tid]; X0[1] = X[3 * tid + 1]; X0[2] = X[3 * tid + 2];
        Z0[0] = Z[2 * tid]; Z0[1] = Z[2 * tid + 1];
    }
    auto edge_in = [&](int e, double (&Xe)[3], double& u, double& v) __attribute__((always_inline)) {
        if (e == tid) {
            Xe[0] = X0[0]; Xe[1] = X0[1]; Xe[2] = X0[2]; u = Z0[0]; v = Z0[1];
        } else {
            Xe[0] = X[3 * e]; Xe[1] = X[3 * e + 1]; Xe[2] = X[3 * e + 2]; u = Z[2 * e]; v = Z[2 * e + 1];
        }
    };

    // linearise at the table S.q / S.t: residuals -> R, per-wave sums -> S.part (then a barrier)
    auto linearise = [&]() __attribute__((always_inline)) {
        double acc[FV];
#pragma unroll
        for (int k = 0; k < FV; ++k) acc[k] = 0.0;
        const double delta = S.delta;
        for (int e = tid; e < O; e += FT) {
            double r0, r1, J[12], Xe[3], u, v;
            edge_in(e, Xe, u, v);
            po_edge(S.q, S.t, Xe, u, v, S.K, r0, r1, J, true);
            R[2 * e] = r0;
            R[2 * e + 1] = r1;
            po_accumulate(r0, r1, J, delta, acc);
        }
        STAMP(24);
        po_rows_to_parts(acc, S, tid);
        STAMP(25);
        lds_barrier();
        STAMP(26);
    };
    // wave 0: the four waves' parts -> S.sum (lane k < FV)
    auto finish_sums = [&]() __attribute__((always_inline)) {
        if (lane < FV) S.sum[lane] = ((S.part[0][lane] + S.part[1][lane]) + S.part[2][lane]) + S.part[3][lane];
        wave_sync();
    };
    auto load_system = [&]() __attribute__((always_inline)) {   // lane 0: S.sum -> H (full symmetric), b
        int k = 0;
        for (int a = 0; a < 6; ++a)
            for (int c = a; c < 6; ++c) { S.H[6 * a + c] = S.sum[k]; S.H[6 * c + a] = S.sum[k]; ++k; }
        for (int a = 0; a < 6; ++a) S.b[a] = S.sum[21 + a];
    };
    // wave 0: (H + lambda D) dx = b, then the candidate pose and its table
    auto solve_step = [&]() __attribute__((always_inline)) {
        double x[6];
        const double lam = S.lam;
        STAMP(30);
        po_ldlt6_lds(S.H, S.b, lam, prm.strategy, S.xs, x);
        STAMP(31);
        double cand[12], q[4], t[3];
        po_pose_add_wave(x, S.pose, S.qp, cand, q, t, lane);
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < 6; ++j) S.dx[j] = x[j];
#pragma unroll
            for (int i = 0; i < 12; ++i) S.cand[i] = cand[i];
#pragma unroll
            for (int i = 0; i < 4; ++i) S.q[i] = q[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) S.t[i] = t[i];
        }
    };

    for (int round = 0; round < 4; ++round) {
        if (tid < 12) S.pose[tid] = pose_in[12 * (size_t)f + tid];   // setEstimate(current_frame_->Pose()) :201
        lds_barrier();
        if (O > 0) {   // Problem::solve returns false with no edge (problem.cpp:157-161)
            if (tid == 0) {
                double q[4], t[3];
                po_table_regs(S.pose, q, t);
                for (int i = 0; i < 4; ++i) { S.q[i] = q[i]; S.qp[i] = q[i]; }
                for (int i = 0; i < 3; ++i) S.t[i] = t[i];
            }
            lds_barrier();
            linearise();
            if (wave == 0) {
                finish_sums();
                if (lane == 0) {
                    load_system();
                    // computeLambdaInitLM (problem.cpp:470-504)
                    S.ni = 2.0;
                    S.chi = 0.5 * S.sum[27];
                    if (prm.strategy == 0) {
                        if (prm.lambda_given) {
                            S.lam = prm.lambda_init;
                        } else {
                            double m = 0.0;
                            for (int i = 0; i < 6; ++i) m = fmax(fabs(S.H[7 * i]), m);
                            S.lam = prm.tau * fmin(prm.lambda_cap, m);
                        }
                    } else {
                        S.lam = 1e-5;
                    }
                    S.last = 1e20;
                    S.iter = 0;
                    S.fc = 0;
                    S.cont = prm.max_iters > 0;
                }
                wave_sync();
                if (S.cont) solve_step();
            }
            lds_barrier();
            while (S.cont) {
                linearise();   // isGoodStepInLM's residuals (:524) and, if accepted, buildHessian's
                if (wave == 0) {
                    finish_sums();
                    if (lane == 0) {
                        // the controller's words into registers first (one batch of LDS loads), the
                        // isGoodStepInLM arithmetic on them, the words back at the end
                        const double tchi = 0.5 * S.sum[27];
                        double lam = S.lam, ni = S.ni, chi = S.chi, last = S.last;
                        int iter = S.iter, fc = S.fc;
                        double dx[6], bv[6], hd[6];
                        for (int i = 0; i < 6; ++i) { dx[i] = S.dx[i]; bv[i] = S.b[i]; hd[i] = S.H[7 * i]; }
                        double scale = 0.0;
                        for (int i = 0; i < 6; ++i)
                            scale += (prm.strategy == 0) ? dx[i] * (lam * dx[i] + bv[i])
                                                         : dx[i] * (lam * hd[i] * dx[i] + bv[i]);
                        scale = 0.5 * scale;
                        scale += 1e-10;
                        const double rho = (chi - tchi) / scale;
                        const bool ok = rho > 0 && isfinite(tchi);
                        if (prm.strategy == 0) {
                            if (ok) {
                                const double m = 2 * rho - 1;
                                double alpha = 1.0 - m * m * m;
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
                        bool inner_end;
                        if (ok) {
                            for (int i = 0; i < 12; ++i) S.pose[i] = S.cand[i];
                            for (int i = 0; i < 4; ++i) S.qp[i] = S.q[i];   // the candidate's table is SE3(pose)'s
                            load_system();
                            inner_end = true;
                        } else {
                            fc += 1;                           // rollbackStates: S.pose untouched
                            inner_end = fc >= prm.max_trials;
                        }
                        int cont = 1;
                        if (inner_end) {
                            iter += 1;
                            if (last - chi < prm.stop_dchi2 || iter >= prm.max_iters) cont = 0;
                            last = chi;
                            fc = 0;
                        }
                        S.lam = lam; S.ni = ni; S.chi = chi; S.last = last; S.iter = iter; S.fc = fc;
                        S.cont = cont;
                    }
                    wave_sync();
                    STAMP(27);
                    if (S.cont) solve_step();
                    STAMP(28);
                }
                lds_barrier();
                STAMP(29);
            }
            its += S.iter;
        }
        // outlier flags (frontend_lego.cpp:205-226); residual_ is "as last evaluated" except for the
        // features already flagged, which are recomputed at the final estimate
        if (tid == 0) {
            double q[4], t[3];
            po_table_regs(S.pose, q, t);
            for (int i = 0; i < 4; ++i) S.q[i] = q[i];
            for (int i = 0; i < 3; ++i) S.t[i] = t[i];
        }
        lds_barrier();
        const double delta = S.delta;
        for (int e = tid; e < O; e += FT) {
            double r0 = R[2 * e], r1 = R[2 * e + 1];
            if (flag[e]) {
                double J[12], Xe[3], u, v;
                edge_in(e, Xe, u, v);
                po_edge(S.q, S.t, Xe, u, v, S.K, r0, r1, J, false);
                R[2 * e] = r0;
                R[2 * e + 1] = r1;
            }
            const double rc = po_rho0(r0, r1, delta);
            flag[e] = rc > 5.991;                       // chi2_th (frontend_lego.cpp:171)
            if (round == 3 && rchi2_out) rchi2_out[o0 + e] = rc;
        }
        lds_barrier();
        if (round == 2 && tid == 0) S.delta = 0.0;     // setCostFunction(nullptr) (:223-225)
        lds_barrier();
    }
    STAMP_FLUSH(24, 8);
    if (tid < 12) pose_out[12 * (size_t)f + tid] = S.pose[tid];
    // inliers: features.size() - cnt_outlier (:249)
    int cnt = 0;
    for (int e = tid; e < O; e += FT) cnt += flag[e] ? 1 : 0;
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
    __shared__ int s_cnt[FT / 64];
    if ((tid & 63) == 0) s_cnt[tid >> 6] = cnt;
    lds_barrier();
    if (tid == 0) {
        int c = 0;
        for (int w = 0; w < FT / 64; ++w) c += s_cnt[w];
        if (inliers_out) inliers_out[f] = O - c;
        if (iters_out) iters_out[f] = its;
    }
}

// dynamic LDS of k_lin<T>: 4 wave scratches + the chunk's pose tables, step and extrinsics
template <int T>
static size_t lin_smem_bytes(int ncam) {
    using Cfg = LinCfg<T>;
    return sizeof(double) * ((size_t)LH_WAVES * Cfg::SCR + 2 * (size_t)Cfg::UMAX * ncam * LH_PT_LDS + Cfg::UMAX * 6 +
                             (size_t)ncam * LH_EXT + (Cfg::UMAX * (Cfg::UMAX + 1) / 2 + 1) / 2 + 1);
}

// ============================================================================
// launchers (host side)
// ============================================================================
extern "C" {


// dynamic LDS of k_lin<T> for ncam cameras (the host rejects windows whose chunks would not fit a CU)
size_t lh_lin_smem(int T, int ncam) {
    switch (T) {
        case 1: return lin_smem_bytes<1>(ncam);
        case 2: return lin_smem_bytes<2>(ncam);
        case 3: return lin_smem_bytes<3>(ncam);
        case 4: return lin_smem_bytes<4>(ncam);
        case 5: return lin_smem_bytes<5>(ncam);
        case 6: return lin_smem_bytes<6>(ncam);
        default: return (size_t)-1;
    }
}

// Raise the dynamic-LDS limit of every k_lin instantiation on the current device (lh_create) to the
// device's per-workgroup LDS (hipDeviceAttributeMaxSharedMemoryPerBlock, read once by the host, which
// also rejects windows whose chunks would exceed it), before any launch.
hipError_t lh_prepare_lin(int lds_limit) {
    const void* fns[] = {reinterpret_cast<const void*>(&k_lin<1, false, false>), reinterpret_cast<const void*>(&k_lin<1, true, false>),
                         reinterpret_cast<const void*>(&k_lin<2, false, false>), reinterpret_cast<const void*>(&k_lin<2, true, false>),
                         reinterpret_cast<const void*>(&k_lin<3, false, false>), reinterpret_cast<const void*>(&k_lin<3, true, false>),
                         reinterpret_cast<const void*>(&k_lin<4, false, false>), reinterpret_cast<const void*>(&k_lin<4, true, false>),
                         reinterpret_cast<const void*>(&k_lin<5, false, false>), reinterpret_cast<const void*>(&k_lin<5, true, false>),
                         reinterpret_cast<const void*>(&k_lin<6, false, false>), reinterpret_cast<const void*>(&k_lin<6, true, false>),
                         reinterpret_cast<const void*>(&k_lin<1, false, true>), reinterpret_cast<const void*>(&k_lin<1, true, true>),
                         reinterpret_cast<const void*>(&k_lin<2, false, true>), reinterpret_cast<const void*>(&k_lin<2, true, true>),
                         reinterpret_cast<const void*>(&k_lin<3, false, true>), reinterpret_cast<const void*>(&k_lin<3, true, true>),
                         reinterpret_cast<const void*>(&k_lin<4, false, true>), reinterpret_cast<const void*>(&k_lin<4, true, true>),
                         reinterpret_cast<const void*>(&k_lin<5, false, true>), reinterpret_cast<const void*>(&k_lin<5, true, true>),
                         reinterpret_cast<const void*>(&k_lin<6, false, true>), reinterpret_cast<const void*>(&k_lin<6, true, true>)};
    for (const void* f : fns) {
        hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds_limit);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t lh_launch_lin(int T, int trial, int nchunks, int chunk_base, hipStream_t st, const lh_chunk* chunks,
                         const lh_subbatch* sbs, const float* obs_uv, const uint32_t* obs_meta, double* rec,
                         double* ptab, const double* ext, const lh_ctrl* ctrl, const double* dxp,
                         double* edge_rho, double* rows, double* csc, const uint32_t* crow, uint8_t* wflag, long nslots,
                         lh_params prm, int nrec, const uint64_t* fixed_bits, double* pose_mat, int writer,
                         lh_reset_args rst) {
    writer = writer ? 1 : 0;   // block 0 stores the trial's candidate poses and tables (the restart, initially)
    if (nchunks + writer <= 0) return hipSuccess;
    dim3 g(nchunks + writer), b(256);
    // (diagnostic) LH_TEST_LIN_LDS_PAD bytes of extra LDS per workgroup: fewer k_lin workgroups per CU, for the
    // latency-hiding probe of scripts/occupancy_probe.py
    static const size_t lds_pad = getenv("LH_TEST_LIN_LDS_PAD") ? (size_t)atol(getenv("LH_TEST_LIN_LDS_PAD")) : 0;
#define LH_LIN(TT, TR)                                                                                             \
    do {                                                                                                           \
        const size_t smem = lin_smem_bytes<TT>(prm.ncam) + lds_pad;                                      \
        if (prm.precision == 1)                                                                                    \
            hipLaunchKernelGGL((k_lin<TT, TR, true>), g, b, smem, st, chunks, sbs, obs_uv, obs_meta, rec, ptab, ext, ctrl, \
                               dxp, edge_rho, rows, csc, crow, wflag, nslots, prm, nrec, fixed_bits, chunk_base,     \
                               pose_mat, writer, rst);                                                             \
        else                                                                                                       \
            hipLaunchKernelGGL((k_lin<TT, TR, false>), g, b, smem, st, chunks, sbs, obs_uv, obs_meta, rec, ptab, ext, ctrl, \
                               dxp, edge_rho, rows, csc, crow, wflag, nslots, prm, nrec, fixed_bits, chunk_base,     \
                               pose_mat, writer, rst);                                                             \
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
        case 10: LH_LIN(5, false); break;
        case 11: LH_LIN(5, true); break;
        case 12: LH_LIN(6, false); break;
        case 13: LH_LIN(6, true); break;
        default: return hipErrorInvalidValue;
    }
#undef LH_LIN
    return hipGetLastError();
}

hipError_t lh_launch_reduce(hipStream_t st, const double* rows, const double* csc, const uint32_t* red_tab, int nred,
                            lh_ctrl* ctrl, double* rs_stage, double* rs_commit, double* maxd,
                            lh_params prm, int n_chunks, int mode, int* host_done, int seq, double* img) {
    hipLaunchKernelGGL(k_reduce, dim3(nred + 1), dim3(RT), 0, st, rows, csc, reinterpret_cast<const uint4*>(red_tab),
                       nred, ctrl, rs_stage, rs_commit, maxd, prm, n_chunks, mode, (volatile int*)host_done, seq, img);
    return hipGetLastError();
}

// k_ctrl's two LDS images (prm.img): zero (the upper triangle where the factor writes L^T, padding
// columns) with the identity on the padding rows [n, ne); k_reduce fills the lower triangle and the rhs
__global__ __launch_bounds__(256) void k_img_init(double* __restrict__ img, int n, int ne) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < 2 * LH_IMG_SZ; i += gridDim.x * 256) {
        const int e = i % LH_IMG_SZ, r = e / LH_IMG_AS, c = e - LH_IMG_AS * r;
        img[i] = (r == c && r >= n && r < ne) ? 1.0 : 0.0;
    }
}

hipError_t lh_launch_img_init(hipStream_t st, double* img, int n) {
    hipLaunchKernelGGL(k_img_init, dim3(64), dim3(256), 0, st, img, n, (n + 15) & ~15);
    return hipGetLastError();
}

hipError_t lh_launch_dense(hipStream_t st, const double* rs_stage, const uint16_t* pair_pq, const lh_ctrl* ctrl,
                           double* gS, int P) {
    if (P <= LH_PMAX) return hipSuccess;
    const int NG = (6 * P + GNB - 1) & ~(GNB - 1);
    hipLaunchKernelGGL(k_dense, dim3(P * (P + 1) / 2), dim3(64), 0, st, rs_stage, pair_pq, ctrl, gS, P, NG);
    return hipGetLastError();
}

hipError_t lh_launch_ctrl(hipStream_t st, lh_ctrl* ctrl, double* rs_commit, const double* rs_stage, const double* maxd,
                          const uint32_t* rsmap, const uint16_t* pair_pq, double* dxp, lh_params prm, int mode,
                          int* host_done, int seq, double* gA, const double* gS, const int32_t* brow_ptr,
                          const uint32_t* brow_ent, const uint16_t* units, lh_band_args band, double* img) {
    const dim3 gl(prm.ladder > 1 ? prm.ladder : 1);   // one workgroup per lambda-ladder rung
    if (prm.P > LH_PMAX && prm.solver == 0 && band.bblk)
    {
        if (prm.band_lu)
            hipLaunchKernelGGL(k_ctrl_b<true>, gl, dim3(CT), 0, st, ctrl, rs_commit, rs_stage, maxd, band.bblk,
                               band.units, band.Lg, band.NDg, dxp, prm, mode, (volatile int*)host_done, seq, img);
        else
            hipLaunchKernelGGL(k_ctrl_b<false>, gl, dim3(CT), 0, st, ctrl, rs_commit, rs_stage, maxd, band.bblk,
                               band.units, band.Lg, band.NDg, dxp, prm, mode, (volatile int*)host_done, seq, img);
    }
    else if (prm.P > LH_PMAX && prm.solver == 1)
        hipLaunchKernelGGL(k_ctrl_p, gl, dim3(CT), 0, st, ctrl, rs_commit, rs_stage, maxd, brow_ptr, brow_ent,
                           dxp, prm, mode, (volatile int*)host_done, seq, gA);   // gA: the PCG's row scratch
    else if (prm.P > LH_PMAX)
        hipLaunchKernelGGL(k_ctrl_g, gl, dim3(GT), 0, st, ctrl, rs_commit, rs_stage, maxd, rsmap,
                           dxp, prm, mode, (volatile int*)host_done, seq, gA, gS);
    else {
        // k_ctrl deciding itself: one more workgroup, the decider of batch chains (ctrl_batch_decider)
        const dim3 gk(gl.x + (prm.dec_in_reduce ? 0 : 1));
        if (prm.solver == 1)
            hipLaunchKernelGGL((k_ctrl<1, false>), gk, dim3(CT), 0, st, ctrl, rs_commit, rs_stage, maxd, pair_pq, units,
                               dxp, prm, mode, (volatile int*)host_done, seq, img);
        else if (prm.img)
            hipLaunchKernelGGL((k_ctrl<0, true>), gk, dim3(CT), 0, st, ctrl, rs_commit, rs_stage, maxd, pair_pq, units,
                               dxp, prm, mode, (volatile int*)host_done, seq, img);
        else
            hipLaunchKernelGGL((k_ctrl<0, false>), gk, dim3(CT), 0, st, ctrl, rs_commit, rs_stage, maxd, pair_pq,
                               units, dxp, prm, mode, (volatile int*)host_done, seq, img);
    }
    return hipGetLastError();
}

// ---- k_gather: results back into window order for the download: landmark positions from the
//      committed records (into out_xyz, pre-filled with the input positions, so landmarks without an
//      edge keep theirs), per-edge rho0 "as last evaluated" from the slots ----
__global__ __launch_bounds__(256) void k_gather(const lh_ctrl* __restrict__ ctrl, const double* __restrict__ rec,
                                                const int32_t* __restrict__ lm_perm, int nrec,
                                                const double* __restrict__ rho, const int32_t* __restrict__ obs_perm,
                                                long nslots, double* __restrict__ out_xyz, double* __restrict__ out_rho) {
    const int cur = __builtin_amdgcn_readfirstlane(ctrl->cur);
    const double* rc = rec + (size_t)cur * nrec * LH_REC;
    const long i0 = (long)blockIdx.x * 256 + threadIdx.x, st = (long)gridDim.x * 256;
    for (long i = i0; i < nslots; i += st) {
        const int o = obs_perm[i];
        if (o >= 0) out_rho[o] = rho[i];
    }
    for (long i = i0; i < 3L * nrec; i += st) {
        const int r = (int)(i / 3), a = (int)(i - 3L * r);
        const int l = lm_perm[r];
        if (l >= 0) out_xyz[3 * (size_t)l + a] = rc[(size_t)r * LH_REC + LH_REC_X + a];
    }
}

hipError_t lh_launch_gather(hipStream_t st, const lh_ctrl* ctrl, const double* rec, const int32_t* lm_perm, int nrec,
                            const double* rho, const int32_t* obs_perm, long nslots, double* out_xyz, double* out_rho) {
    const long n = std::max(nslots, 3L * nrec);
    if (n <= 0) return hipSuccess;
    const int blocks = (int)std::max(1L, std::min(4096L, (n + 255) / 256));
    hipLaunchKernelGGL(k_gather, dim3(blocks), dim3(256), 0, st, ctrl, rec, lm_perm, nrec, rho, obs_perm, nslots,
                       out_xyz, out_rho);
    return hipGetLastError();
}

// ---- Backend::Optimize's outlier pass (backend_lego.cpp:163-194) on the device, over rho0 as last
//      evaluated (d_rho, slot order).  The loop counts edges with rho0 > th for th = th0 2^k, k < 5 (the
//      thresholds it can visit: doubling is exact), so one pass counts all five, as per-block partials
//      (integers: the same totals in any order, and no counter to zero first); the second pass sums the
//      partials, replays the loop on the totals and writes one flag per edge in window order, with the
//      threshold and the counts behind the flags, so one copy brings all of it back. ----
#define LH_OCB 256   // blocks of the counting pass
__global__ __launch_bounds__(256) void k_outlier_count(const double* __restrict__ rho, const int32_t* __restrict__ obs_perm,
                                                       long nslots, double th0, unsigned* __restrict__ part) {
    __shared__ unsigned wsum[4][5];
    unsigned c[5] = {0u, 0u, 0u, 0u, 0u};
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nslots; i += (long)gridDim.x * 256) {
        if (obs_perm[i] < 0) continue;   // padding slot
        const double r = rho[i];
        double th = th0;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            c[k] += (r > th) ? 1u : 0u;   // a NaN rho0 counts as an inlier, as in the reference
            th *= 2;
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        unsigned v = c[k];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) wsum[wave][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < 5)
        part[blockIdx.x * 5 + threadIdx.x] = wsum[0][threadIdx.x] + wsum[1][threadIdx.x] + wsum[2][threadIdx.x] + wsum[3][threadIdx.x];
}

// A sharded window's pass (the reference counts the whole window's edges): the counting blocks' partials summed
// into this rank's {5 counts, its edge count} as doubles (exact below 2^53), which the handle's exchange sums
// over the ranks before k_outlier_flags reads them (gtot)
__global__ __launch_bounds__(64) void k_outlier_total(const unsigned* __restrict__ part, int nparts, long n_obs,
                                                      double* __restrict__ tot) {
    long c[5] = {0, 0, 0, 0, 0};
    for (int b = threadIdx.x; b < nparts; b += 64)
#pragma unroll
        for (int k = 0; k < 5; ++k) c[k] += part[b * 5 + k];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        long v = c[k];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (threadIdx.x == 0) tot[k] = (double)v;
    }
    if (threadIdx.x == 0) tot[5] = (double)n_obs;
}

__global__ __launch_bounds__(256) void k_outlier_flags(const double* __restrict__ rho, const int32_t* __restrict__ obs_perm,
                                                       long nslots, long n_obs, double th0, const unsigned* __restrict__ part,
                                                       int nparts, uint8_t* __restrict__ flags, double* __restrict__ res,
                                                       const double* __restrict__ gtot) {
    __shared__ long tot[5];
    if (gtot) {   // the all-ranks totals (k_outlier_total + the exchange)
        if (threadIdx.x < 5) tot[threadIdx.x] = (long)gtot[threadIdx.x];
        n_obs = (long)gtot[5];
    } else if (threadIdx.x < 64) {
        long c[5] = {0, 0, 0, 0, 0};
        for (int b = threadIdx.x; b < nparts; b += 64)
#pragma unroll
            for (int k = 0; k < 5; ++k) c[k] += part[b * 5 + k];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            long v = c[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if (threadIdx.x == 0) tot[k] = v;
        }
    }
    __syncthreads();
    // backend_lego.cpp:164-184, on the totals (every thread the same)
    double th = th0;
    long cin = 0, cout = 0;
    for (int it = 0; it < 5; ++it) {
        cout = tot[it];
        cin = n_obs - cout;
        const double ratio = cin / double(cin + cout);
        if (ratio > 0.5) break;
        th *= 2;
    }
    const long i0 = (long)blockIdx.x * 256 + threadIdx.x, st = (long)gridDim.x * 256;
    for (long i = i0; i < nslots; i += st) {   // :186-194
        const int o = obs_perm[i];
        if (o >= 0) flags[o] = rho[i] > th ? 1 : 0;
    }
    if (i0 == 0) {
        res[0] = th;
        res[1] = (double)cin;
        res[2] = (double)cout;
    }
}

// ---- the one-shot peer-write exchange (LH_COMM_P2P, lh_common.h) ----
// Block d writes this rank's partial (the packed reduced system, and max|diag H_ll| at the initial linearisation)
// into slot `rank` of rank d's buffer, then its arrival tag.  The buffers are plain device memory mapped over IPC,
// whose caches are not coherent with another agent's: the data goes out as system-scope stores and is read back as
// system-scope loads (no stale line in either GPU's L2), every thread's stores are fenced at system scope before
// the block's barrier, and thread 0 stores the tag with a system-scope release.
__global__ __launch_bounds__(1024) void k_p2p_push(const double* __restrict__ src, const double* __restrict__ maxd,
                                                   int n, lh_peers peers, int rank, int world, int parity,
                                                   unsigned long long tag, long slot) {
    const int d = blockIdx.x;
    double* dst = peers.p[d] + ((size_t)parity * world + rank) * slot;
    for (int i = threadIdx.x; i < n; i += 1024) __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (threadIdx.x == 0) __hip_atomic_store(dst + n, maxd ? *maxd : 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long* tags = reinterpret_cast<unsigned long long*>(peers.p[d] + (size_t)2 * world * slot);
        __hip_atomic_store(tags + parity * world + rank, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Every block waits for the trial's tags of all ranks in this rank's buffer (system-scope acquire; a bounded
// wait: past ~4 s the exchange is declared failed in *err, a host-mapped word, and the block exits), then sums
// its elements over the slots in rank order into the reduced system (max for max|diag H_ll|): every rank gets the
// same bits.
__global__ __launch_bounds__(256) void k_p2p_sum(double* __restrict__ dst, double* __restrict__ maxd, int n,
                                                 const double* __restrict__ buf, int world, int parity,
                                                 unsigned long long tag, long slot, int mode, volatile int* err) {
    __shared__ int s_ok;
    if (threadIdx.x == 0) {
        const unsigned long long* tags = reinterpret_cast<const unsigned long long*>(buf + (size_t)2 * world * slot) +
                                         parity * world;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
        int ok = *err ? 0 : 1;   // (an earlier exchange of this handle failed: no second wait)
        for (int r = 0; r < world && ok; ++r)
            while (__hip_atomic_load(tags + r, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != tag) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) { ok = 0; *err = 1; break; }
                __builtin_amdgcn_s_sleep(2);
            }
        s_ok = ok;
    }
    __syncthreads();
    if (!s_ok) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const double* src = buf + (size_t)parity * world * slot;
    auto ld = [](const double* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        double v = ld(src + i);
        for (int r = 1; r < world; ++r) v += ld(src + (size_t)r * slot + i);
        dst[i] = v;
    }
    if (mode == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
        double m = ld(src + n);
        for (int r = 1; r < world; ++r) m = fmax(m, ld(src + (size_t)r * slot + n));
        *maxd = m;
    }
}

hipError_t lh_launch_p2p(hipStream_t st, double* rs, double* maxd, int n, lh_peers peers, int rank, int world,
                         int parity, unsigned long long tag, long slot, int mode, int* err) {
    if (world < 1 || world > LH_P2P_MAX || (long)n + 1 > slot) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_p2p_push, dim3(world), dim3(1024), 0, st, (const double*)rs, mode == 0 ? (const double*)maxd : nullptr,
                       n, peers, rank, world, parity, tag, slot);
    const int nb = std::max(1, std::min(32, (n + 255) / 256));
    hipLaunchKernelGGL(k_p2p_sum, dim3(nb), dim3(256), 0, st, rs, maxd, n, (const double*)peers.p[rank], world, parity,
                       tag, slot, mode, (volatile int*)err);
    return hipGetLastError();
}

// part: LH_OCB * 5 counters; flags: n_obs bytes, then (16-byte aligned) the threshold and the two counts
hipError_t lh_launch_outliers(hipStream_t st, const double* rho, const int32_t* obs_perm, long nslots, long n_obs,
                              double th0, unsigned* part, uint8_t* flags) {
    if (nslots <= 0) return hipSuccess;
    const int nb_c = (int)std::max(1L, std::min((long)LH_OCB, (nslots + 255) / 256));
    const int nb_f = (int)std::max(1L, std::min(2048L, (nslots + 255) / 256));
    double* res = reinterpret_cast<double*>(flags + ((n_obs + 15) & ~15L));
    hipLaunchKernelGGL(k_outlier_count, dim3(nb_c), dim3(256), 0, st, rho, obs_perm, nslots, th0, part);
    hipLaunchKernelGGL(k_outlier_flags, dim3(nb_f), dim3(256), 0, st, rho, obs_perm, nslots, n_obs, th0,
                       (const unsigned*)part, nb_c, flags, res, (const double*)nullptr);
    return hipGetLastError();
}

// the sharded pass in two halves around the exchange of tot[6] (this rank's counts and edge count)
hipError_t lh_launch_outlier_counts(hipStream_t st, const double* rho, const int32_t* obs_perm, long nslots, long n_obs,
                                    double th0, unsigned* part, double* tot) {
    const int nb_c = (int)std::max(1L, std::min((long)LH_OCB, (nslots + 255) / 256));
    if (nslots > 0) hipLaunchKernelGGL(k_outlier_count, dim3(nb_c), dim3(256), 0, st, rho, obs_perm, nslots, th0, part);
    hipLaunchKernelGGL(k_outlier_total, dim3(1), dim3(64), 0, st, (const unsigned*)part, nslots > 0 ? nb_c : 0, n_obs, tot);
    return hipGetLastError();
}

hipError_t lh_launch_outlier_flags(hipStream_t st, const double* rho, const int32_t* obs_perm, long nslots, long n_obs,
                                   double th0, const double* gtot, uint8_t* flags) {
    const int nb_f = (int)std::max(1L, std::min(2048L, (nslots + 255) / 256));
    double* res = reinterpret_cast<double*>(flags + ((n_obs + 15) & ~15L));
    hipLaunchKernelGGL(k_outlier_flags, dim3(nb_f), dim3(256), 0, st, rho, obs_perm, nslots, n_obs, th0,
                       (const unsigned*)nullptr, 0, flags, res, gtot);
    return hipGetLastError();
}

// ---- LDL^T probe (tests): x = (S)^-1 b through k_ctrl's LDS layout and lds_ldlt_solve (natural
//      order, a dense envelope) or lds_pcg_solve, for a dense symmetric S (row-major n x n, n <= LH_NPAD) ----
__global__ __launch_bounds__(CT) void k_ldlt_probe(const double* __restrict__ S, const double* __restrict__ b, int n,
                                                   double* __restrict__ x, int solver, double tol, int max_it,
                                                   int* __restrict__ iters) {
    __shared__ double A[(NP + 1) * AS];
    __shared__ __attribute__((aligned(16))) double dg[NP];
    __shared__ __attribute__((aligned(16))) double xsol[NP];
    __shared__ uint16_t s_units[16 * LH_NSTEP];
    const int tid = threadIdx.x, NE = (n + 15) & ~15;
    if (tid == 0) {
        int32_t fcb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int order[15] = LH_ORDER_CTRL;
        lh_ctrl_units(n, fcb, order, 15, LH_NSTEP, s_units);
    }
    for (int e = tid; e < NE * NE; e += CT) {
        const int r = e / NE, c = e - NE * (e / NE);
        if (c <= r) A[r * AS + c] = (r < n) ? ((c < n) ? S[(size_t)r * n + c] : 0.0) : (r == c ? 1.0 : 0.0);
        else A[r * AS + c] = 0.0;
    }
    if (tid < NE) A[NP * AS + tid] = tid < n ? b[tid] : 0.0;
    lds_barrier();
    if (solver == 1) {
        __shared__ __attribute__((aligned(16))) double s_pcg[48];
        const int its = lds_pcg_solve(A, xsol, dg, s_pcg, n, tid, tol, (max_it > 0 ? max_it : 2 * n) + 1);
        if (tid == 0 && iters) *iters = its;
    } else {
        lds_ldlt_solve(A, xsol, n, NE, tid, nullptr, s_units);
    }
    lds_barrier();
    if (tid < n) x[tid] = xsol[tid];
}

// ---- the same probe through k_ctrl_g's global-memory solve (LH_NPAD < n <= 6 LH_PMAX_WIN):
//      gA: scratch of ceil32(n)^2 doubles ----
__global__ __launch_bounds__(GT) void k_ldlt_g_probe(const double* __restrict__ S, const double* __restrict__ b, int n,
                                                     double* __restrict__ x, double* __restrict__ gA) {
    __shared__ double pnl[GNMAX * GPS];
    __shared__ double dg[GNMAX], yv[GNMAX];
    __shared__ int perm[GNMAX], iperm[GNMAX];
    const int tid = threadIdx.x, NG = (n + GNB - 1) & ~(GNB - 1);
    for (int i = tid; i < n; i += GT) dg[i] = S[(size_t)i * n + i];
    lds_barrier();
    for (int row = tid; row < n; row += GT) {
        double di = fabs(dg[row]);
        if (!(di == di)) di = -1.0;
        int r = 0;
        for (int j = 0; j < n; ++j) {
            double d = fabs(dg[j]);
            if (!(d == d)) d = -1.0;
            r += (d > di) || (d == di && j < row);
        }
        perm[r] = row;
        iperm[row] = r;
    }
    lds_barrier();
    const bool all_zero = !(fabs(dg[perm[0]]) > 0.0);
    lds_barrier();
    if (all_zero)
        for (int i = tid; i < n; i += GT) { perm[i] = i; iperm[i] = i; }
    lds_barrier();
    for (int x2 = tid; x2 < NG * NG; x2 += GT) {
        const int r = x2 / NG, c = x2 - NG * (x2 / NG);
        double v = 0.0;
        if (r < n && c < n) v = (c <= r) ? S[(size_t)perm[r] * n + perm[c]] : 0.0;
        else if (r == c) v = 1.0;
        gA[x2] = v;
    }
    for (int i = tid; i < NG; i += GT) yv[i] = i < n ? b[perm[i]] : 0.0;
    __syncthreads();
    g_ldlt_solve(gA, NG, n, all_zero, yv, pnl);
    for (int i = tid; i < n; i += GT) x[perm[i]] = yv[i];
}

hipError_t lh_launch_ldlt_g_probe(const double* S, const double* b, int n, double* x, double* gA) {
    hipLaunchKernelGGL(k_ldlt_g_probe, dim3(1), dim3(GT), 0, 0, S, b, n, x, gA);
    return hipGetLastError();
}

hipError_t lh_launch_ldlt_probe(const double* S, const double* b, int n, double* x, int solver, double tol, int max_it,
                                int* iters) {
    if (n < 1 || n > LH_NPAD) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ldlt_probe, dim3(1), dim3(CT), 0, 0, S, b, n, x, solver, tol, max_it, iters);
    return hipGetLastError();
}

// ---- empty kernel: the HIP-event bracket floor of one launch (bench.py's roofline timing) ----
__global__ void k_nop() {}

hipError_t lh_launch_nop(hipStream_t st) {
    hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, st);
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
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(lh_stamps), sizeof(unsigned long long) * (n < 256 ? n : 256));
    if (e != hipSuccess) return e;
    if (reset) {
        unsigned long long z[256] = {0};
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

hipError_t lh_launch_frames(hipStream_t st, int n_frames, const int64_t* obs_ptr, const double* pose_in,
                            const double* pts, const double* uv, const uint8_t* flag_in, lh_params prm, double* res,
                            double* pose_out, uint8_t* flag_out, double* rchi2_out, int32_t* iters_out,
                            int32_t* inliers_out) {
    if (n_frames <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_frames, dim3(n_frames), dim3(FT), 0, st, obs_ptr, pose_in, pts, uv, flag_in, prm, res, pose_out,
                       flag_out, rchi2_out, iters_out, inliers_out);
    return hipGetLastError();
}

}  // extern "C"

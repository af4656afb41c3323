/*
 * lego_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference
 * LEGO-SLAM backend solve (lego::Problem in SLAM mode driven by
 * Backend::Optimize).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this file; the product never links it.
 *
 * PARITY UNPINNED: the reference cannot be compiled here (Eigen3, Sophus,
 * OpenCV, glog are absent) and its only test
 * (test/legoslam_test_triangulation.cpp) is off this path, so no reference
 * output pins this restatement.  It is cross-checked against an independent
 * NumPy twin (oracle/lego_oracle_np.py) and against known-answer tests.
 *
 * Two variants with identical per-edge arithmetic and LM logic:
 *   variant 0  "ref_dense":  literal — dense n x n H, dense Hmm_inv, dense
 *              tempH = Hpm * Hmm_inv, LDLT of the reduced system.
 *              (problem.cpp:273-358, :380-430).  Small windows only.
 *   variant 1  "ref_sparse": block-sparse — per-landmark H_ll, per-pose H_pp,
 *              per-(landmark,pose) H_pl, per-landmark Schur; OpenMP over
 *              landmarks with a fixed-order reduction.  The CPU baseline.
 *
 * Third-party arithmetic restated (versions unpinned in the reference):
 *   Eigen  Quaternion(Matrix3), toRotationMatrix, _transformVector, quaternion
 *          product; PartialPivLU inverse (problem.cpp:399); LDLT with
 *          diagonal pivoting and its pseudo-inverse solve (problem.cpp:420).
 *   Sophus SE3(Matrix4), SE3::exp, SE3 * SE3, SO3 renormalisation (Sophus 1.0).
 * Evaluation order follows the reference expressions; compile with
 * -ffp-contract=off (the reference's x86-64 build has no FMA).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct orc_options {
    int32_t max_iters;     /* solve(10)              backend_lego.cpp:161 */
    int32_t max_trials;    /* false_cnt_threshold    problem.cpp:178      */
    int32_t strategy;      /* 0 DEFAULT, 1 STRATEGY1 problem.h:45-50      */
    int32_t verbose;
    int32_t n_threads;     /* ref_sparse OpenMP threads (0 = runtime default) */
    int32_t gate_mode;     /* 0: reference Huber gate (rho1 + 2 rho2 e2 > 0.0, base_edge.cpp:55);
                              1: diagnostic only - treat the analytically-zero residue as 0 */
    double huber_delta;    /* 5.991; <= 0: no cost function */
    double stop_dchi2;     /* 1e-5 */
    double tau;            /* 1e-5 */
    double lambda_cap;     /* 5e10 */
    double lambda_init;    /* < 0 computed */
    int32_t linear_solver; /* 0 Eigen LDLT (problem.cpp:420); 1 PCG (PCGSolver :584-614, fixed) */
    int32_t pcg_max_iters; /* <= 0: 2 * rows (problem.cpp:422) */
    double pcg_tol;        /* 1e-6 (problem.cpp:597) */
    int32_t degenerate_guard; /* 0: reference (problem.cpp:396-400: the LU inverse of a rank-deficient
                                 H_ll as it comes); 1: the solver's opt-in guard (include/lego_ba.h):
                                 a landmark with < 2 edges or a non-PD H_ll is held fixed (no Schur
                                 term, dx_l = 0) - restated here so the guard mode is checked too */
    int32_t pad_;
} orc_options;

typedef struct orc_stats {
    double chi2_initial, chi2_final, lambda_final, time_ms;
    int32_t iterations, trials, accepted, trace_len;
    int32_t pcg_iterations, pad_;
} orc_stats;

/* ======================= Eigen / Sophus restatements ======================= */

/* Eigen::Quaternion from rotation matrix (quaternionbase_assign_impl<.,3,3>).
   q = {w, x, y, z}; R row-major. */
static void q_from_R(const double *R, double q[4]) {
#define M(i, j) R[3 * (i) + (j)]
    double t = M(0, 0) + M(1, 1) + M(2, 2);
    if (t > 0.0) {
        t = sqrt(t + 1.0);
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
        t = sqrt(M(i, i) - M(j, j) - M(k, k) + 1.0);
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

/* Eigen QuaternionBase::toRotationMatrix */
static void R_from_q(const double q[4], double *R) {
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;          R[2] = txz + twy;
    R[3] = txy + twz;          R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;          R[7] = tyz + twx;          R[8] = 1.0 - (txx + tyy);
}

static void cross3(const double a[3], const double b[3], double c[3]) {
    double c0 = a[1] * b[2] - a[2] * b[1];
    double c1 = a[2] * b[0] - a[0] * b[2];
    double c2 = a[0] * b[1] - a[1] * b[0];
    c[0] = c0; c[1] = c1; c[2] = c2;
}

/* Eigen QuaternionBase::_transformVector */
static void q_rotate(const double q[4], const double v[3], double out[3]) {
    double uv[3], uv2[3];
    cross3(q + 1, v, uv);
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    cross3(q + 1, uv, uv2);
    for (int i = 0; i < 3; ++i) out[i] = v[i] + q[0] * uv[i] + uv2[i];
}

/* Eigen quaternion product + Sophus SO3Base::operator*= renormalisation */
static void q_mul(const double a[4], const double b[4], double o[4]) {
    double w = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    double x = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    double y = a[0] * b[2] + a[2] * b[0] + a[3] * b[1] - a[1] * b[3];
    double z = a[0] * b[3] + a[3] * b[0] + a[1] * b[2] - a[2] * b[1];
    double sq = w * w + x * x + y * y + z * z;
    if (sq != 1.0) {
        double s = 2.0 / (1.0 + sq);
        w *= s; x *= s; y *= s; z *= s;
    }
    o[0] = w; o[1] = x; o[2] = y; o[3] = z;
}

typedef struct { double q[4]; double t[3]; } se3_t;

/* Sophus SE3(Matrix4): estimate_ is the 4x4 (here row-major [R|t], 12 doubles) */
static void se3_from_mat(const double *T12, se3_t *T) {
    double R[9] = {T12[0], T12[1], T12[2], T12[4], T12[5], T12[6], T12[8], T12[9], T12[10]};
    q_from_R(R, T->q);
    T->t[0] = T12[3]; T->t[1] = T12[7]; T->t[2] = T12[11];
}
/* SE3::matrix() */
static void se3_to_mat(const se3_t *T, double *T12) {
    double R[9];
    R_from_q(T->q, R);
    for (int i = 0; i < 3; ++i) {
        T12[4 * i] = R[3 * i]; T12[4 * i + 1] = R[3 * i + 1]; T12[4 * i + 2] = R[3 * i + 2];
        T12[4 * i + 3] = T->t[i];
    }
}
/* SE3 * SE3: (so3*so3, t + so3*t') */
static void se3_mul(const se3_t *A, const se3_t *B, se3_t *C) {
    se3_t r;
    double rt[3];
    q_mul(A->q, B->q, r.q);
    q_rotate(A->q, B->t, rt);
    for (int i = 0; i < 3; ++i) r.t[i] = A->t[i] + rt[i];
    *C = r;
}
/* SE3 * point */
static void se3_apply(const se3_t *T, const double X[3], double Y[3]) {
    double r[3];
    q_rotate(T->q, X, r);
    for (int i = 0; i < 3; ++i) Y[i] = r[i] + T->t[i];
}

/* Sophus SE3::exp, twist a = (upsilon[3] translation, omega[3] rotation) */
static void se3_exp(const double a[6], se3_t *T) {
    const double eps = 1e-10; /* Sophus Constants<double>::epsilon() */
    const double *w = a + 3;
    double theta_sq = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double theta = sqrt(theta_sq);
    double half_theta = 0.5 * theta;
    double imag, real;
    if (theta < eps) {
        double theta_po4 = theta_sq * theta_sq;
        imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_po4;
        real = 1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * theta_po4;
    } else {
        double s = sin(half_theta);
        imag = s / theta;
        real = cos(half_theta);
    }
    T->q[0] = real; T->q[1] = imag * w[0]; T->q[2] = imag * w[1]; T->q[3] = imag * w[2];
    double V[9];
    if (theta < eps) {
        R_from_q(T->q, V);
    } else {
        double Om[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
        double Om2[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                Om2[3 * i + j] = Om[3 * i] * Om[j] + Om[3 * i + 1] * Om[3 + j] + Om[3 * i + 2] * Om[6 + j];
        double c1 = (1.0 - cos(theta)) / theta_sq;
        double c2 = (theta - sin(theta)) / (theta_sq * theta);
        for (int i = 0; i < 9; ++i) V[i] = ((i % 4 == 0) ? 1.0 : 0.0) + c1 * Om[i] + c2 * Om2[i];
    }
    for (int i = 0; i < 3; ++i) T->t[i] = V[3 * i] * a[0] + V[3 * i + 1] * a[1] + V[3 * i + 2] * a[2];
}

/* Eigen PartialPivLU(3x3).inverse() (dynamic-size block inverse, problem.cpp:399).
   A, Ainv row-major 3x3. */
static void lu_inverse3(const double *A, double *Ainv) {
    double lu[9];
    int tr[3];
    memcpy(lu, A, sizeof(lu));
    for (int k = 0; k < 3; ++k) {
        int piv = k;
        double big = fabs(lu[3 * k + k]);
        for (int i = k + 1; i < 3; ++i)
            if (fabs(lu[3 * i + k]) > big) { big = fabs(lu[3 * i + k]); piv = i; }
        tr[k] = piv;
        if (big != 0.0) {
            if (piv != k)
                for (int j = 0; j < 3; ++j) { double t = lu[3 * k + j]; lu[3 * k + j] = lu[3 * piv + j]; lu[3 * piv + j] = t; }
            for (int i = k + 1; i < 3; ++i) lu[3 * i + k] /= lu[3 * k + k];
        }
        for (int i = k + 1; i < 3; ++i)
            for (int j = k + 1; j < 3; ++j) lu[3 * i + j] -= lu[3 * i + k] * lu[3 * k + j];
    }
    /* dst = P * I */
    double X[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int k = 0; k < 3; ++k)
        if (tr[k] != k)
            for (int j = 0; j < 3; ++j) { double t = X[3 * k + j]; X[3 * k + j] = X[3 * tr[k] + j]; X[3 * tr[k] + j] = t; }
    /* unit-lower forward substitution, column-oriented */
    for (int k = 0; k < 3; ++k)
        for (int i = k + 1; i < 3; ++i)
            for (int j = 0; j < 3; ++j) X[3 * i + j] -= lu[3 * i + k] * X[3 * k + j];
    /* upper back substitution */
    for (int k = 2; k >= 0; --k) {
        for (int j = 0; j < 3; ++j) X[3 * k + j] /= lu[3 * k + k];
        for (int i = 0; i < k; ++i)
            for (int j = 0; j < 3; ++j) X[3 * i + j] -= lu[3 * i + k] * X[3 * k + j];
    }
    memcpy(Ainv, X, sizeof(X));
}

/* Eigen LDLT<Lower> (ldlt_inplace::unblocked, diagonal pivoting) followed by
   LDLT::_solve_impl.  A is n x n row-major (lower triangle used), destroyed. */
static void ldlt_solve(double *A, int n, const double *b, double *x) {
    int *tr = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    double *temp = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
#define A_(i, j) A[(size_t)(i) * (size_t)n + (size_t)(j)]
    int all_zero = 0;
    for (int k = 0; k < n; ++k) {
        int idx = k;
        double big = fabs(A_(k, k));
        for (int i = k + 1; i < n; ++i)
            if (fabs(A_(i, i)) > big) { big = fabs(A_(i, i)); idx = i; }
        tr[k] = idx;
        if (k != idx) {
            for (int j = 0; j < k; ++j) { double t = A_(k, j); A_(k, j) = A_(idx, j); A_(idx, j) = t; }
            for (int i = idx + 1; i < n; ++i) { double t = A_(i, k); A_(i, k) = A_(i, idx); A_(i, idx) = t; }
            { double t = A_(k, k); A_(k, k) = A_(idx, idx); A_(idx, idx) = t; }
            for (int i = k + 1; i < idx; ++i) { double t = A_(i, k); A_(i, k) = A_(idx, i); A_(idx, i) = t; }
        }
        int rs = n - k - 1;
        if (k > 0) {
            for (int j = 0; j < k; ++j) temp[j] = A_(j, j) * A_(k, j);
            double s = 0.0;
            for (int j = 0; j < k; ++j) s += A_(k, j) * temp[j];
            A_(k, k) -= s;
            for (int i = k + 1; i < n; ++i) {
                double si = 0.0;
                for (int j = 0; j < k; ++j) si += A_(i, j) * temp[j];
                A_(i, k) -= si;
            }
        }
        double akk = A_(k, k);
        int valid = fabs(akk) > 0.0;
        if (k == 0 && !valid) {
            for (int j = 0; j < n; ++j) tr[j] = j;
            all_zero = 1;
            break;
        }
        if (rs > 0 && valid)
            for (int i = k + 1; i < n; ++i) A_(i, k) /= akk;
    }
    (void)all_zero;   /* Eigen records it (ret = false) but LDLT::_solve_impl still runs both solves */
    /* LDLT::_solve_impl: dst = P b; L^-1; pseudo-inverse of D; L^-T; P^T.  The triangular solves
       follow Eigen's triangular_solve_vector in NaN/Inf semantics (for finite data the operations
       below are bitwise those of a plain column-oriented solve, since x - L*0 == x):
       - L (unit lower, column-major storage): panels of 8 rows; inside a panel a column whose x
         is exactly 0 is skipped (not_equal_strict(rhs[i], 0)); rows below the panel take the
         whole panel by GEMV, zero entries included (0 * NaN = NaN there);
       - L^T (unit upper, row-major view): dot products, nothing skipped.
       After an all-NaN S (an inf PartialPivLU inverse makes every S entry NaN through the dense
       GEMMs, problem.cpp:399-404) this leaves a NaN step, not the zero step a shortcut would. */
    for (int i = 0; i < n; ++i) x[i] = b[i];
    for (int k = 0; k < n; ++k) { int j = tr[k]; if (j != k) { double t = x[k]; x[k] = x[j]; x[j] = t; } }
    for (int p0 = 0; p0 < n; p0 += 8) {
        const int p1 = p0 + 8 < n ? p0 + 8 : n;
        for (int k = p0; k < p1; ++k) {
            if (x[k] != 0.0)
                for (int i = k + 1; i < p1; ++i) x[i] -= A_(i, k) * x[k];
            for (int i = p1; i < n; ++i) x[i] -= A_(i, k) * x[k];
        }
    }
    const double tol = 2.2250738585072014e-308; /* numeric_limits<double>::min() */
    for (int i = 0; i < n; ++i) {
        double d = A_(i, i);
        if (fabs(d) > tol) x[i] /= d; else x[i] = 0.0;
    }
    for (int k = n - 1; k >= 0; --k)
        for (int i = 0; i < k; ++i) x[i] -= A_(k, i) * x[k];
    for (int k = n - 1; k >= 0; --k) { int j = tr[k]; if (j != k) { double t = x[k]; x[k] = x[j]; x[j] = t; } }
#undef A_
    free(tr);
    free(temp);
}

/* Problem::PCGSolver (problem.cpp:584-614), the Jacobi-PCG the reference left commented out at
   :421-422 (called there with maxIter = 2 * rows), restated with its bug fixed: the reference
   computes the first step alpha * p but never adds it to x (:595-596).  Same stop rule
   (||r|| > 1e-6 ||b||, :597-598), same update order.  A zero diagonal entry preconditions with 0
   (Eigen's inverse would give inf and a NaN step).  A is read through its lower triangle.
   Returns the number of steps (the reference's first step plus its loop iterations). */
static int pcg_solve(const double *A, int n, const double *b, double *x, double tol, int max_iters) {
#define AL_(i, j) ((i) >= (j) ? A[(size_t)(i) * (size_t)n + (size_t)(j)] : A[(size_t)(j) * (size_t)n + (size_t)(i)])
    const int maxit = max_iters > 0 ? max_iters : 2 * n;
    double *minv = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    double *r = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    double *z = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    double *p = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    double *w = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    double rz = 0.0, bb = 0.0;
    for (int i = 0; i < n; ++i) {
        const double d = AL_(i, i);
        minv[i] = d != 0.0 ? 1.0 / d : 0.0;
        x[i] = 0.0;
        r[i] = b[i];
        z[i] = minv[i] * r[i];
        p[i] = z[i];
        rz += r[i] * z[i];
        bb += r[i] * r[i];
    }
    const double thr = tol * sqrt(bb);
    int steps = 0;
    if (bb > 0.0) {
        for (;;) {
            double pw = 0.0;
            for (int i = 0; i < n; ++i) {
                double s = 0.0;
                for (int j = 0; j < n; ++j) s += AL_(i, j) * p[j];
                w[i] = s;
                pw += p[i] * s;
            }
            const double alpha = rz / pw;
            double rr = 0.0, rzn = 0.0;
            for (int i = 0; i < n; ++i) {
                x[i] += alpha * p[i];
                r[i] -= alpha * w[i];
                z[i] = minv[i] * r[i];
                rr += r[i] * r[i];
                rzn += r[i] * z[i];
            }
            ++steps;
            if (!(sqrt(rr) > thr) || steps >= maxit + 1) break;
            const double beta = rzn / rz;
            rz = rzn;
            for (int i = 0; i < n; ++i) p[i] = beta * p[i] + z[i];
        }
    }
    free(minv); free(r); free(z); free(p); free(w);
#undef AL_
    return steps;
}

/* The reduced pose solve: Eigen LDLT (the reference) or the fixed PCG (its commented-out option). */
static int reduced_solve(const orc_options *o, double *S, int n, const double *bs, double *x) {
    if (o->linear_solver == 1) return pcg_solve(S, n, bs, x, o->pcg_tol, o->pcg_max_iters);
    ldlt_solve(S, n, bs, x);
    return 0;
}

/* ============================ problem state ============================== */

typedef struct {
    /* inputs */
    int32_t P, L, ncam, variant;
    int64_t O;
    const uint8_t *fixed;
    const uint32_t *op, *ol;
    const uint8_t *oc;
    const double *uv;
    double K[4];
    se3_t *ext;
    orc_options opt;
    /* state: estimate_ and estimate_backup_ */
    double *pose, *pose_bak; /* P x 12 */
    double *lm, *lm_bak;     /* L x 3  */
    /* per edge (residual_ as last computed, Jacobians, robust weights) */
    double *res;             /* O x 2 */
    /* linearisation */
    double *H, *b;           /* dense: n x n, n */
    double *Hpp, *bp;        /* sparse: P x 36, P x 6 */
    double *Hll, *bl;        /* L x 9, L x 3 */
    double *Hpl;             /* per edge 6x3 (row-major) */
    double *dx;              /* n */
    double *hdiag;           /* n: diag of Hessian_ (lambda init, STRATEGY1) */
    /* landmark-major edge order */
    int64_t *lm_ptr, *lm_edges;
    int64_t n;
    double chi, lambda, ni;
    /* orc_reduced_system: capture the undamped reduced system instead of solving */
    double *S_out, *bs_out;
    int64_t pcg_iters;       /* PCG steps summed over the solve's trials */
    int64_t *lm_cnt;         /* edges per landmark (degenerate_guard) */
} prob_t;

/* degenerate_guard 1: the solver's test (lh_kernels.hip k_lin): fewer than two edges, or a Cholesky
   pivot of H_ll that is not positive */
static int hll_degenerate(const prob_t *pb, int32_t l, const double *H) {
    if (pb->lm_cnt[l] < 2) return 1;
    if (!(H[0] > 0.0)) return 1;
    const double l00 = sqrt(H[0]), l10 = H[1] / l00, l20 = H[2] / l00;
    const double a11 = H[4] - l10 * l10;
    if (!(a11 > 0.0)) return 1;
    const double l21 = (H[5] - l20 * l10) / sqrt(a11);
    const double a22 = H[8] - l20 * l20 - l21 * l21;
    return !(a22 > 0.0) || !isfinite(a22);
}

/* ---- EdgeProjection arithmetic (include/legoslam/lego_types.h:200-254) ---- */

static void edge_residual(const prob_t *pb, int64_t e, double r[2]) {
    se3_t T;
    se3_from_mat(pb->pose + 12 * (size_t)pb->op[e], &T);
    const double *X = pb->lm + 3 * (size_t)pb->ol[e];
    int c = pb->oc ? pb->oc[e] : 0;
    double Pb[3], Pc[3];
    se3_apply(&T, X, Pb);             /* T * X                 */
    se3_apply(&pb->ext[c], Pb, Pc);   /* _cam_ext * (T * X)    */
    const double fx = pb->K[0], fy = pb->K[1], cx = pb->K[2], cy = pb->K[3];
    double p0 = fx * Pc[0] + 0.0 * Pc[1] + cx * Pc[2]; /* _K * Pc, row by row */
    double p1 = 0.0 * Pc[0] + fy * Pc[1] + cy * Pc[2];
    double p2 = 0.0 * Pc[0] + 0.0 * Pc[1] + 1.0 * Pc[2];
    double den = p2 + 1e-18;                          /* pos_pixel /= (z + 1e-18) */
    p0 /= den; p1 /= den;
    r[0] = pb->uv[2 * e] - p0;                        /* measurement_ - pos_pixel */
    r[1] = pb->uv[2 * e + 1] - p1;
}

static void edge_jacobians(const prob_t *pb, int64_t e, double Jp[12], double Jl[6]) {
    se3_t T, ET;
    se3_from_mat(pb->pose + 12 * (size_t)pb->op[e], &T);
    int c = pb->oc ? pb->oc[e] : 0;
    const double *X = pb->lm + 3 * (size_t)pb->ol[e];
    se3_mul(&pb->ext[c], &T, &ET);    /* _cam_ext * T * pw: (ext*T)*pw */
    double Pc[3];
    se3_apply(&ET, X, Pc);
    const double fx = pb->K[0], fy = pb->K[1];
    const double x = Pc[0], y = Pc[1], z = Pc[2];
    const double zi = 1.0 / (z + 1e-18);
    const double zi2 = zi * zi;
    Jp[0] = -fx * zi;             Jp[1] = 0.0;              Jp[2] = fx * x * zi2;
    Jp[3] = fx * x * y * zi2;     Jp[4] = -fx - fx * x * x * zi2; Jp[5] = fx * y * zi;
    Jp[6] = 0.0;                  Jp[7] = -fy * zi;         Jp[8] = fy * y * zi2;
    Jp[9] = fy + fy * y * y * zi2; Jp[10] = -fy * x * y * zi2; Jp[11] = -fy * x * zi;
    /* j_j = j_i(:, 0:3) * ext.rotationMatrix() * T.rotationMatrix() */
    double Re[9], Rt[9], A[6];
    R_from_q(pb->ext[c].q, Re);
    R_from_q(T.q, Rt);
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j)
            A[3 * i + j] = Jp[6 * i] * Re[j] + Jp[6 * i + 1] * Re[3 + j] + Jp[6 * i + 2] * Re[6 + j];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j)
            Jl[3 * i + j] = A[3 * i] * Rt[j] + A[3 * i + 1] * Rt[3 + j] + A[3 * i + 2] * Rt[6 + j];
}

/* HuberCost::compute (cost_function.cpp:5-17) */
static void huber(double delta, double e2, double rho[3]) {
    double d2 = delta * delta;
    if (e2 <= d2) { rho[0] = e2; rho[1] = 1.0; rho[2] = 0.0; }
    else {
        double s = sqrt(e2);
        rho[0] = 2 * s * delta - d2;
        rho[1] = delta / s;
        rho[2] = -0.5 * rho[1] / e2;
    }
}

/* BaseEdge::getRobustChi2 (base_edge.cpp:33-42) */
static double robust_chi2(const prob_t *pb, const double r[2]) {
    double e2 = r[0] * r[0] + r[1] * r[1]; /* r^T * I * r */
    if (pb->opt.huber_delta > 0) { double rho[3]; huber(pb->opt.huber_delta, e2, rho); return rho[0]; }
    return e2;
}

/* BaseEdge::computeRobustInformation (base_edge.cpp:44-64); W row-major 2x2 */
static void robust_info(const prob_t *pb, const double r[2], double W[4], double *drho) {
    if (pb->opt.huber_delta > 0) {
        double e2 = r[0] * r[0] + r[1] * r[1];
        double rho[3];
        huber(pb->opt.huber_delta, e2, rho);
        W[0] = rho[1]; W[1] = 0.0; W[2] = 0.0; W[3] = rho[1];
        if (rho[1] + 2 * rho[2] * e2 > 0.0 && !(pb->opt.gate_mode == 1 && e2 > pb->opt.huber_delta * pb->opt.huber_delta)) {
            double s = 2 * rho[2];
            W[0] += s * r[0] * r[0]; W[1] += s * r[0] * r[1];
            W[2] += s * r[1] * r[0]; W[3] += s * r[1] * r[1];
        }
        *drho = rho[1];
    } else {
        W[0] = 1.0; W[1] = 0.0; W[2] = 0.0; W[3] = 1.0;
        *drho = 1.0;
    }
}

/* hessian = (J_i^T W) J_j for J_i (2 x di), J_j (2 x dj); out di x dj row-major */
static void jtwj(const double *Ji, int di, const double W[4], const double *Jj, int dj, double *out) {
    double JtW[12];
    for (int a = 0; a < di; ++a)
        for (int m = 0; m < 2; ++m) JtW[2 * a + m] = Ji[a] * W[m] + Ji[di + a] * W[2 + m];
    for (int a = 0; a < di; ++a)
        for (int c = 0; c < dj; ++c) out[dj * a + c] = JtW[2 * a] * Jj[c] + JtW[2 * a + 1] * Jj[dj + c];
}

/* per-edge linearisation pieces shared by both variants */
typedef struct { double Hpp[36], Hpl[18], Hll[9], bp[6], bl[3]; } edge_lin_t;

static void edge_linearize(prob_t *pb, int64_t e, edge_lin_t *E) {
    double r[2], Jp[12], Jl[6], W[4], drho;
    edge_residual(pb, e, r);
    pb->res[2 * e] = r[0];
    pb->res[2 * e + 1] = r[1];
    edge_jacobians(pb, e, Jp, Jl);
    robust_info(pb, r, W, &drho);
    int pf = pb->fixed && pb->fixed[pb->op[e]];
    memset(E, 0, sizeof(*E));
    if (!pf) {
        jtwj(Jp, 6, W, Jp, 6, E->Hpp);
        jtwj(Jp, 6, W, Jl, 3, E->Hpl);
        for (int a = 0; a < 6; ++a) E->bp[a] = -((drho * Jp[a]) * r[0] + (drho * Jp[6 + a]) * r[1]);
    }
    jtwj(Jl, 3, W, Jl, 3, E->Hll);
    for (int a = 0; a < 3; ++a) E->bl[a] = -((drho * Jl[a]) * r[0] + (drho * Jl[3 + a]) * r[1]);
}

/* ================================ dense ================================== */

static void build_dense(prob_t *pb) {
    const int64_t n = pb->n;
    const int64_t np = 6 * (int64_t)pb->P;
    memset(pb->H, 0, sizeof(double) * (size_t)(n * n));
    memset(pb->b, 0, sizeof(double) * (size_t)n);
    for (int64_t e = 0; e < pb->O; ++e) {
        edge_lin_t E;
        edge_linearize(pb, e, &E);
        int64_t ip = 6 * (int64_t)pb->op[e], il = np + 3 * (int64_t)pb->ol[e];
        for (int a = 0; a < 6; ++a)
            for (int c = 0; c < 6; ++c) pb->H[(ip + a) * n + ip + c] += E.Hpp[6 * a + c];
        for (int a = 0; a < 6; ++a)
            for (int c = 0; c < 3; ++c) {
                pb->H[(ip + a) * n + il + c] += E.Hpl[3 * a + c];
                pb->H[(il + c) * n + ip + a] += E.Hpl[3 * a + c];
            }
        for (int a = 0; a < 3; ++a)
            for (int c = 0; c < 3; ++c) pb->H[(il + a) * n + il + c] += E.Hll[3 * a + c];
        for (int a = 0; a < 6; ++a) pb->b[ip + a] += E.bp[a];
        for (int a = 0; a < 3; ++a) pb->b[il + a] += E.bl[a];
    }
    for (int64_t i = 0; i < n; ++i) pb->hdiag[i] = pb->H[i * n + i];
}

static void solve_dense(prob_t *pb) {
    const int64_t n = pb->n, np = 6 * (int64_t)pb->P, nm = n - np;
    double *Hmm_inv = (double *)calloc((size_t)(nm * nm), sizeof(double));
    for (int32_t l = 0; l < pb->L; ++l) {
        double blk[9], inv[9];
        int64_t o = np + 3 * (int64_t)l;
        for (int a = 0; a < 3; ++a)
            for (int c = 0; c < 3; ++c) blk[3 * a + c] = pb->H[(o + a) * n + o + c];
        lu_inverse3(blk, inv);
        if (pb->opt.degenerate_guard && hll_degenerate(pb, l, blk))
            for (int a = 0; a < 9; ++a) inv[a] = 0.0;   /* held fixed: no Schur term, dx_l = 0 */
        for (int a = 0; a < 3; ++a)
            for (int c = 0; c < 3; ++c) Hmm_inv[(3 * l + a) * nm + 3 * l + c] = inv[3 * a + c];
    }
    /* tempH = Hpm * Hmm_inv */
    double *tempH = (double *)calloc((size_t)(np * nm), sizeof(double));
    for (int64_t i = 0; i < np; ++i)
        for (int64_t k = 0; k < nm; ++k) {
            double h = pb->H[i * n + np + k];
            for (int64_t j = 0; j < nm; ++j) tempH[i * nm + j] += h * Hmm_inv[k * nm + j];
        }
    /* S = Hpp - tempH * Hmp; bs = bpp - tempH * bmm */
    double *S = (double *)malloc(sizeof(double) * (size_t)(np * np));
    double *bs = (double *)malloc(sizeof(double) * (size_t)np);
    for (int64_t i = 0; i < np; ++i) {
        for (int64_t j = 0; j < np; ++j) {
            double s = 0.0;
            for (int64_t k = 0; k < nm; ++k) s += tempH[i * nm + k] * pb->H[(np + k) * n + j];
            S[i * np + j] = pb->H[i * n + j] - s;
        }
        double s = 0.0;
        for (int64_t k = 0; k < nm; ++k) s += tempH[i * nm + k] * pb->b[np + k];
        bs[i] = pb->b[i] - s;
    }
    for (int64_t i = 0; i < np; ++i) {
        if (pb->opt.strategy == 0) S[i * np + i] += pb->lambda;
        else S[i * np + i] += pb->lambda * S[i * np + i];
    }
    pb->pcg_iters += reduced_solve(&pb->opt, S, (int)np, bs, pb->dx);
    /* dxl = Hmm_inv * (bmm - Hmp * dxp) */
    double *tmp = (double *)malloc(sizeof(double) * (size_t)(nm > 0 ? nm : 1));
    for (int64_t k = 0; k < nm; ++k) {
        double s = 0.0;
        for (int64_t j = 0; j < np; ++j) s += pb->H[(np + k) * n + j] * pb->dx[j];
        tmp[k] = pb->b[np + k] - s;
    }
    for (int64_t k = 0; k < nm; ++k) {
        double s = 0.0;
        for (int64_t j = 0; j < nm; ++j) s += Hmm_inv[k * nm + j] * tmp[j];
        pb->dx[np + k] = s;
    }
    free(tmp); free(S); free(bs); free(tempH); free(Hmm_inv);
}

/* ================================ sparse ================================= */

static int nthreads(const prob_t *pb) {
#ifdef _OPENMP
    return pb->opt.n_threads > 0 ? pb->opt.n_threads : omp_get_max_threads();
#else
    (void)pb;
    return 1;
#endif
}

static void build_sparse(prob_t *pb) {
    const int32_t P = pb->P;
    const int nt = nthreads(pb);
    double *part = (double *)calloc((size_t)nt * (size_t)P * 42, sizeof(double));
#pragma omp parallel num_threads(nt)
    {
#ifdef _OPENMP
        int tid = omp_get_thread_num();
#else
        int tid = 0;
#endif
        double *myHpp = part + (size_t)tid * (size_t)P * 42;
        double *mybp = myHpp + (size_t)P * 36;
#pragma omp for schedule(static)
        for (int32_t l = 0; l < pb->L; ++l) {
            double Hll[9] = {0}, bl[3] = {0};
            for (int64_t q = pb->lm_ptr[l]; q < pb->lm_ptr[l + 1]; ++q) {
                int64_t e = pb->lm_edges[q];
                edge_lin_t E;
                edge_linearize(pb, e, &E);
                uint32_t p = pb->op[e];
                for (int a = 0; a < 36; ++a) myHpp[36 * (size_t)p + a] += E.Hpp[a];
                for (int a = 0; a < 6; ++a) mybp[6 * (size_t)p + a] += E.bp[a];
                for (int a = 0; a < 9; ++a) Hll[a] += E.Hll[a];
                for (int a = 0; a < 3; ++a) bl[a] += E.bl[a];
                memcpy(pb->Hpl + 18 * (size_t)e, E.Hpl, sizeof(E.Hpl));
            }
            memcpy(pb->Hll + 9 * (size_t)l, Hll, sizeof(Hll));
            memcpy(pb->bl + 3 * (size_t)l, bl, sizeof(bl));
        }
    }
    memset(pb->Hpp, 0, sizeof(double) * (size_t)P * 36);
    memset(pb->bp, 0, sizeof(double) * (size_t)P * 6);
    for (int t = 0; t < nt; ++t) {
        const double *h = part + (size_t)t * (size_t)P * 42;
        for (size_t a = 0; a < (size_t)P * 36; ++a) pb->Hpp[a] += h[a];
        for (size_t a = 0; a < (size_t)P * 6; ++a) pb->bp[a] += h[(size_t)P * 36 + a];
    }
    free(part);
    for (int32_t p = 0; p < P; ++p)
        for (int a = 0; a < 6; ++a) {
            pb->hdiag[6 * p + a] = pb->Hpp[36 * p + 7 * a];
            pb->b[6 * p + a] = pb->bp[6 * p + a];
        }
    for (int32_t l = 0; l < pb->L; ++l)
        for (int a = 0; a < 3; ++a) {
            pb->hdiag[6 * (int64_t)P + 3 * l + a] = pb->Hll[9 * (size_t)l + 4 * a];
            pb->b[6 * (int64_t)P + 3 * l + a] = pb->bl[3 * (size_t)l + a];
        }
}

static void solve_sparse(prob_t *pb) {
    const int32_t P = pb->P;
    const int64_t np = 6 * (int64_t)P;
    const int nt = nthreads(pb);
    double *part = (double *)calloc((size_t)nt * (size_t)(np * np + np), sizeof(double));
    double *Hinv = (double *)malloc(sizeof(double) * 9 * (size_t)(pb->L > 0 ? pb->L : 1));
#pragma omp parallel num_threads(nt)
    {
#ifdef _OPENMP
        int tid = omp_get_thread_num();
#else
        int tid = 0;
#endif
        double *myS = part + (size_t)tid * (size_t)(np * np + np);
        double *mybs = myS + np * np;
        double Hpl[64 * 18];
        int32_t pose_of[64];
#pragma omp for schedule(static)
        for (int32_t l = 0; l < pb->L; ++l) {
            double *inv = Hinv + 9 * (size_t)l;
            lu_inverse3(pb->Hll + 9 * (size_t)l, inv);
            if (pb->opt.degenerate_guard && hll_degenerate(pb, l, pb->Hll + 9 * (size_t)l))
                for (int a = 0; a < 9; ++a) inv[a] = 0.0;   /* held fixed: no Schur term, dx_l = 0 */
            /* merge the landmark's edges per pose: H_pl block of the dense H */
            int nb = 0;
            for (int64_t q = pb->lm_ptr[l]; q < pb->lm_ptr[l + 1]; ++q) {
                int64_t e = pb->lm_edges[q];
                int32_t p = (int32_t)pb->op[e];
                if (nb > 0 && pose_of[nb - 1] == p) {
                    for (int a = 0; a < 18; ++a) Hpl[18 * (nb - 1) + a] += pb->Hpl[18 * (size_t)e + a];
                } else if (nb < 64) {
                    pose_of[nb] = p;
                    memcpy(Hpl + 18 * nb, pb->Hpl + 18 * (size_t)e, 18 * sizeof(double));
                    ++nb;
                }
            }
            const double *bl = pb->bl + 3 * (size_t)l;
            for (int i = 0; i < nb; ++i) {
                double tH[18]; /* tempH block: Hpl_i * Hll^-1 */
                for (int a = 0; a < 6; ++a)
                    for (int c = 0; c < 3; ++c)
                        tH[3 * a + c] = Hpl[18 * i + 3 * a] * inv[c] + Hpl[18 * i + 3 * a + 1] * inv[3 + c] +
                                        Hpl[18 * i + 3 * a + 2] * inv[6 + c];
                int64_t pi = 6 * (int64_t)pose_of[i];
                for (int j = 0; j < nb; ++j) {
                    int64_t pj = 6 * (int64_t)pose_of[j];
                    for (int a = 0; a < 6; ++a)
                        for (int c = 0; c < 6; ++c)
                            myS[(pi + a) * np + pj + c] += tH[3 * a] * Hpl[18 * j + 3 * c] +
                                                           tH[3 * a + 1] * Hpl[18 * j + 3 * c + 1] +
                                                           tH[3 * a + 2] * Hpl[18 * j + 3 * c + 2];
                }
                for (int a = 0; a < 6; ++a) mybs[pi + a] += tH[3 * a] * bl[0] + tH[3 * a + 1] * bl[1] + tH[3 * a + 2] * bl[2];
            }
        }
    }
    double *S = (double *)malloc(sizeof(double) * (size_t)(np * np));
    double *bs = (double *)malloc(sizeof(double) * (size_t)np);
    for (int64_t i = 0; i < np * np; ++i) S[i] = 0.0;
    for (int64_t i = 0; i < np; ++i) bs[i] = 0.0;
    for (int t = 0; t < nt; ++t) {
        const double *s = part + (size_t)t * (size_t)(np * np + np);
        for (int64_t i = 0; i < np * np; ++i) S[i] += s[i];
        for (int64_t i = 0; i < np; ++i) bs[i] += s[np * np + i];
    }
    free(part);
    for (int32_t p = 0; p < P; ++p)
        for (int a = 0; a < 6; ++a)
            for (int c = 0; c < 6; ++c) S[(6 * p + a) * np + 6 * p + c] = pb->Hpp[36 * p + 6 * a + c] - S[(6 * p + a) * np + 6 * p + c];
    for (int64_t i = 0; i < np; ++i)
        for (int64_t j = 0; j < np; ++j)
            if (i / 6 != j / 6) S[i * np + j] = -S[i * np + j];
    for (int64_t i = 0; i < np; ++i) bs[i] = pb->bp[i] - bs[i];
    if (pb->S_out) {   /* orc_reduced_system */
        memcpy(pb->S_out, S, sizeof(double) * (size_t)(np * np));
        memcpy(pb->bs_out, bs, sizeof(double) * (size_t)np);
        free(S); free(bs); free(Hinv);
        return;
    }
    for (int64_t i = 0; i < np; ++i) {
        if (pb->opt.strategy == 0) S[i * np + i] += pb->lambda;
        else S[i * np + i] += pb->lambda * S[i * np + i];
    }
    pb->pcg_iters += reduced_solve(&pb->opt, S, (int)np, bs, pb->dx);
    free(S); free(bs);
    /* back substitution: dxl = Hll^-1 (bl - Hlp * dxp) */
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int32_t l = 0; l < pb->L; ++l) {
        double t[3];
        for (int a = 0; a < 3; ++a) {
            double s = 0.0;
            for (int64_t q = pb->lm_ptr[l]; q < pb->lm_ptr[l + 1]; ++q) {
                int64_t e = pb->lm_edges[q];
                const double *h = pb->Hpl + 18 * (size_t)e;
                const double *d = pb->dx + 6 * (size_t)pb->op[e];
                for (int c = 0; c < 6; ++c) s += h[3 * c + a] * d[c];
            }
            t[a] = pb->bl[3 * (size_t)l + a] - s;
        }
        const double *inv = Hinv + 9 * (size_t)l;
        for (int a = 0; a < 3; ++a)
            pb->dx[np + 3 * (int64_t)l + a] = inv[3 * a] * t[0] + inv[3 * a + 1] * t[1] + inv[3 * a + 2] * t[2];
    }
    free(Hinv);
}

/* =============================== LM driver =============================== */

static void build_hessian(prob_t *pb) {
    if (pb->variant == 0) build_dense(pb); else build_sparse(pb);
    memset(pb->dx, 0, sizeof(double) * (size_t)pb->n); /* delta_x_ = 0 (problem.cpp:357) */
}

static void solve_linear(prob_t *pb) {
    if (pb->variant == 0) solve_dense(pb); else solve_sparse(pb);
}

/* Problem::updateStates (problem.cpp:433-455) with VertexPose::add / VertexXYZ::add */
static void update_states(prob_t *pb) {
    memcpy(pb->pose_bak, pb->pose, sizeof(double) * 12 * (size_t)pb->P);
    memcpy(pb->lm_bak, pb->lm, sizeof(double) * 3 * (size_t)pb->L);
    for (int32_t p = 0; p < pb->P; ++p) {
        const double *d = pb->dx + 6 * (size_t)p;
        double u[6];
        int bad = 0;
        for (int a = 0; a < 6; ++a) if (isnan(d[a]) || isinf(d[a])) bad = 1;
        for (int a = 0; a < 6; ++a) u[a] = bad ? 0.0 : d[a];
        se3_t E, T, R;
        se3_exp(u, &E);
        se3_from_mat(pb->pose + 12 * (size_t)p, &T);
        se3_mul(&E, &T, &R);
        se3_to_mat(&R, pb->pose + 12 * (size_t)p);
    }
    const int64_t np = 6 * (int64_t)pb->P;
#pragma omp parallel for schedule(static) num_threads(nthreads(pb))
    for (int32_t l = 0; l < pb->L; ++l) {
        const double *d = pb->dx + np + 3 * (int64_t)l;
        if (!isnan(d[0]) && !isnan(d[1]) && !isnan(d[2]) && !isinf(d[0]) && !isinf(d[1]) && !isinf(d[2])) {
            pb->lm[3 * (size_t)l] += d[0];
            pb->lm[3 * (size_t)l + 1] += d[1];
            pb->lm[3 * (size_t)l + 2] += d[2];
        }
    }
}

static void rollback_states(prob_t *pb) {
    memcpy(pb->pose, pb->pose_bak, sizeof(double) * 12 * (size_t)pb->P);
    memcpy(pb->lm, pb->lm_bak, sizeof(double) * 3 * (size_t)pb->L);
}

/* sum of robust chi2 over the current residuals, fixed order */
static double sum_rchi2(prob_t *pb, int recompute) {
    const int nt = pb->variant == 0 ? 1 : nthreads(pb);
    double *part = (double *)calloc((size_t)nt, sizeof(double));
#pragma omp parallel num_threads(nt)
    {
#ifdef _OPENMP
        int tid = omp_get_thread_num();
#else
        int tid = 0;
#endif
        double s = 0.0;
#pragma omp for schedule(static)
        for (int64_t e = 0; e < pb->O; ++e) {
            if (recompute) edge_residual(pb, e, pb->res + 2 * e);
            s += robust_chi2(pb, pb->res + 2 * e);
        }
        part[tid] = s;
    }
    double s = 0.0;
    for (int t = 0; t < nt; ++t) s += part[t];
    free(part);
    return s;
}

static void lambda_init(prob_t *pb) {
    pb->ni = 2.0;
    pb->lambda = -1.0;
    pb->chi = 0.5 * sum_rchi2(pb, 0);
    if (pb->opt.strategy == 0) {
        if (pb->opt.lambda_init < 0) {
            double m = 0.0;
            for (int64_t i = 0; i < pb->n; ++i) m = fmax(fabs(pb->hdiag[i]), m);
            m = fmin(pb->opt.lambda_cap, m);
            pb->lambda = pb->opt.tau * m;
        } else {
            pb->lambda = pb->opt.lambda_init;
        }
    } else {
        pb->lambda = 1e-5;
    }
}

static int good_step(prob_t *pb) {
    double temp_chi = 0.5 * sum_rchi2(pb, 1);
    if (pb->opt.strategy == 0) {
        double scale = 0.0;
        for (int64_t i = 0; i < pb->n; ++i) scale += pb->dx[i] * (pb->lambda * pb->dx[i] + pb->b[i]);
        scale = 0.5 * scale;
        scale += 1e-10;
        double rho = (pb->chi - temp_chi) / scale;
        if (pb->opt.verbose >= 2) printf("trial rho %.17g chi %.17g tchi %.17g lambda %.17g\n", rho, pb->chi, temp_chi, pb->lambda);
        if (rho > 0 && isfinite(temp_chi)) {
            double alpha = 1.0 - pow((2 * rho - 1), 3);
            alpha = fmin(alpha, 2.0 / 3.0);
            double f = fmax(1.0 / 3.0, alpha);
            pb->lambda *= f;
            pb->ni = 2;
            pb->chi = temp_chi;
            return 1;
        }
        pb->lambda *= pb->ni;
        pb->ni *= 2;
        return 0;
    } else {
        double scale = 0.0;
        for (int64_t i = 0; i < pb->n; ++i) scale += pb->dx[i] * (pb->lambda * pb->hdiag[i] * pb->dx[i] + pb->b[i]);
        scale = 0.5 * scale;
        scale += 1e-10;
        double rho = (pb->chi - temp_chi) / scale;
        if (pb->opt.verbose >= 2) printf("trial rho %.17g chi %.17g tchi %.17g lambda %.17g\n", rho, pb->chi, temp_chi, pb->lambda);
        if (rho > 0 && isfinite(temp_chi)) {
            pb->lambda = fmax(pb->lambda / 9.0, 1e-7);
            pb->chi = temp_chi;
            return 1;
        }
        pb->lambda = fmin(pb->lambda * 11.0, 1e7);
        return 0;
    }
}

typedef struct { const uint32_t *ol, *op; } sort_ctx_t;
static const sort_ctx_t *g_sort_ctx;
static int cmp_edge_q(const void *a, const void *b) {
    int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    const sort_ctx_t *c = g_sort_ctx;
    if (c->ol[x] != c->ol[y]) return c->ol[x] < c->ol[y] ? -1 : 1;
    if (c->op[x] != c->op[y]) return c->op[x] < c->op[y] ? -1 : 1;
    return x < y ? -1 : (x > y);
}

double orc_now_ms(void);

/*
 * orc_solve — Backend::Optimize's problem.solve(max_iters) on one window.
 * Returns 0 on success, 1 for an empty problem (problem.cpp:157-161),
 * 2 for bad arguments.
 */
static int orc_run(int variant, int32_t P, const double *pose_in, const uint8_t *fixed,
                   int32_t L, const double *lm_in, int64_t O, const uint32_t *op, const uint32_t *ol,
                   const uint8_t *oc, const double *uv, const double *K, int32_t ncam, const double *cam_ext,
                   const orc_options *opt, double *pose_out, double *lm_out, double *edge_rchi2,
                   double *trace_chi, double *trace_lambda, int32_t trace_cap, orc_stats *st,
                   double *S_out, double *bs_out, double *chi2_out) {
    memset(st, 0, sizeof(*st));
    if (P < 0 || L < 0 || O < 0) return 2;
    if (O == 0 || (P + L) == 0) return 1;
    for (int64_t e = 0; e < O; ++e) {
        if (op[e] >= (uint32_t)P || ol[e] >= (uint32_t)L) return 2;
        if (oc && oc[e] >= (uint8_t)(ncam > 0 ? ncam : 1)) return 2;
    }
    double t0 = orc_now_ms();
    prob_t pb;
    memset(&pb, 0, sizeof(pb));
    pb.P = P; pb.L = L; pb.O = O; pb.variant = variant;
    pb.fixed = fixed; pb.op = op; pb.ol = ol; pb.oc = oc; pb.uv = uv;
    memcpy(pb.K, K, sizeof(pb.K));
    pb.opt = *opt;
    int nc = ncam > 0 ? ncam : 1;
    pb.ext = (se3_t *)malloc(sizeof(se3_t) * (size_t)nc);
    for (int c = 0; c < nc; ++c) {
        if (cam_ext && ncam > 0) se3_from_mat(cam_ext + 12 * c, &pb.ext[c]);
        else { double I12[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0}; se3_from_mat(I12, &pb.ext[c]); }
    }
    pb.n = 6 * (int64_t)P + 3 * (int64_t)L;
    pb.pose = (double *)malloc(sizeof(double) * 12 * (size_t)P);
    pb.pose_bak = (double *)malloc(sizeof(double) * 12 * (size_t)P);
    pb.lm = (double *)malloc(sizeof(double) * 3 * (size_t)(L > 0 ? L : 1));
    pb.lm_bak = (double *)malloc(sizeof(double) * 3 * (size_t)(L > 0 ? L : 1));
    memcpy(pb.pose, pose_in, sizeof(double) * 12 * (size_t)P);
    memcpy(pb.lm, lm_in, sizeof(double) * 3 * (size_t)L);
    pb.res = (double *)calloc(2 * (size_t)O, sizeof(double));
    pb.lm_cnt = (int64_t *)calloc((size_t)(L > 0 ? L : 1), sizeof(int64_t));
    for (int64_t e = 0; e < O; ++e) pb.lm_cnt[ol[e]]++;
    pb.dx = (double *)calloc((size_t)pb.n, sizeof(double));
    pb.b = (double *)calloc((size_t)pb.n, sizeof(double));
    pb.hdiag = (double *)calloc((size_t)pb.n, sizeof(double));
    if (variant == 0) {
        pb.H = (double *)malloc(sizeof(double) * (size_t)(pb.n * pb.n));
    } else {
        pb.Hpp = (double *)malloc(sizeof(double) * 36 * (size_t)P);
        pb.bp = (double *)malloc(sizeof(double) * 6 * (size_t)P);
        pb.Hll = (double *)malloc(sizeof(double) * 9 * (size_t)(L > 0 ? L : 1));
        pb.bl = (double *)malloc(sizeof(double) * 3 * (size_t)(L > 0 ? L : 1));
        pb.Hpl = (double *)malloc(sizeof(double) * 18 * (size_t)O);
        pb.lm_ptr = (int64_t *)calloc((size_t)L + 1, sizeof(int64_t));
        pb.lm_edges = (int64_t *)malloc(sizeof(int64_t) * (size_t)O);
        for (int64_t e = 0; e < O; ++e) pb.lm_edges[e] = e;
        sort_ctx_t sc = {ol, op};
        g_sort_ctx = &sc;
        qsort(pb.lm_edges, (size_t)O, sizeof(int64_t), cmp_edge_q);
        for (int64_t e = 0; e < O; ++e) pb.lm_ptr[ol[e] + 1]++;
        for (int32_t l = 0; l < L; ++l) pb.lm_ptr[l + 1] += pb.lm_ptr[l];
    }

    /* ---- Problem::solve (problem.cpp:156-230) ---- */
    if (S_out) {   /* orc_reduced_system: linearise at the input state, reduce, stop */
        pb.S_out = S_out;
        pb.bs_out = bs_out;
        build_hessian(&pb);
        *chi2_out = sum_rchi2(&pb, 0);   /* sum of rho0 (not halved) */
        solve_linear(&pb);
        free(pb.ext); free(pb.pose); free(pb.pose_bak); free(pb.lm); free(pb.lm_bak);
        free(pb.res); free(pb.dx); free(pb.b); free(pb.hdiag);
        free(pb.H); free(pb.Hpp); free(pb.bp); free(pb.Hll); free(pb.bl); free(pb.Hpl);
        free(pb.lm_ptr); free(pb.lm_edges); free(pb.lm_cnt);
        return 0;
    }
    if (pb.opt.verbose) printf("==========LEGO OPTIMIZER==========\n");
    build_hessian(&pb);
    lambda_init(&pb);
    st->chi2_initial = pb.chi;
    int stop = 0, iter = 0;
    double last_chi = 1e20;
    while (!stop && iter < pb.opt.max_iters) {
        if (pb.opt.verbose) printf("Iteration = %d,\tChi = %g,\tLambda = %g\n", iter, pb.chi, pb.lambda);
        if (st->trace_len < trace_cap) {
            if (trace_chi) trace_chi[st->trace_len] = pb.chi;
            if (trace_lambda) trace_lambda[st->trace_len] = pb.lambda;
        }
        st->trace_len++;
        int ok = 0, false_cnt = 0;
        while (!ok && false_cnt < pb.opt.max_trials) {
            solve_linear(&pb);
            update_states(&pb);
            ok = good_step(&pb);
            st->trials++;
            if (ok) { build_hessian(&pb); false_cnt = 0; st->accepted++; }
            else { false_cnt++; rollback_states(&pb); }
        }
        ++iter;
        if (last_chi - pb.chi < pb.opt.stop_dchi2) {
            if (pb.opt.verbose) printf("\nStop the optimization: [last_chi_(%g) - currentChi_(%g) = %g] < %g\n",
                                        last_chi, pb.chi, last_chi - pb.chi, pb.opt.stop_dchi2);
            stop = 1;
        }
        last_chi = pb.chi;
    }
    st->iterations = iter;
    st->chi2_final = pb.chi;
    st->lambda_final = pb.lambda;
    st->pcg_iterations = (int32_t)pb.pcg_iters;
    if (st->trace_len > trace_cap) st->trace_len = trace_cap;

    if (pose_out) memcpy(pose_out, pb.pose, sizeof(double) * 12 * (size_t)P);
    if (lm_out) memcpy(lm_out, pb.lm, sizeof(double) * 3 * (size_t)L);
    if (edge_rchi2)
        for (int64_t e = 0; e < O; ++e) edge_rchi2[e] = robust_chi2(&pb, pb.res + 2 * e);
    st->time_ms = orc_now_ms() - t0;

    free(pb.ext); free(pb.pose); free(pb.pose_bak); free(pb.lm); free(pb.lm_bak);
    free(pb.res); free(pb.dx); free(pb.b); free(pb.hdiag);
    free(pb.H); free(pb.Hpp); free(pb.bp); free(pb.Hll); free(pb.bl); free(pb.Hpl);
    free(pb.lm_ptr); free(pb.lm_edges); free(pb.lm_cnt);
    return 0;
}

int orc_solve(int variant, int32_t P, const double *pose_in, const uint8_t *fixed,
              int32_t L, const double *lm_in, int64_t O, const uint32_t *op, const uint32_t *ol,
              const uint8_t *oc, const double *uv, const double *K, int32_t ncam, const double *cam_ext,
              const orc_options *opt, double *pose_out, double *lm_out, double *edge_rchi2,
              double *trace_chi, double *trace_lambda, int32_t trace_cap, orc_stats *st) {
    return orc_run(variant, P, pose_in, fixed, L, lm_in, O, op, ol, oc, uv, K, ncam, cam_ext, opt, pose_out, lm_out,
                   edge_rchi2, trace_chi, trace_lambda, trace_cap, st, NULL, NULL, NULL);
}

/*
 * orc_reduced_system — the undamped reduced pose system of one window at its input state:
 * S = H_pp - H_pl H_ll^-1 H_lp (6P x 6P, row-major, full), bs = b_p - H_pl H_ll^-1 b_l
 * (problem.cpp:382-405 without the lambda of :406-418), chi2 = sum rho0.  Landmark shards
 * contribute additively: the sum over shards equals the full window (the multi-GPU path's
 * one all-reduce).  Block-sparse variant only.
 */
int orc_reduced_system(int32_t P, const double *pose_in, const uint8_t *fixed, int32_t L, const double *lm_in,
                       int64_t O, const uint32_t *op, const uint32_t *ol, const uint8_t *oc, const double *uv,
                       const double *K, int32_t ncam, const double *cam_ext, const orc_options *opt,
                       double *S_out, double *bs_out, double *chi2_out) {
    orc_stats st;
    if (!S_out || !bs_out || !chi2_out) return 2;
    return orc_run(1, P, pose_in, fixed, L, lm_in, O, op, ol, oc, uv, K, ncam, cam_ext, opt, NULL, NULL, NULL,
                   NULL, NULL, 0, &st, S_out, bs_out, chi2_out);
}

#include <time.h>
double orc_now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

/* ---- small exports for known-answer tests ---- */
void orc_se3_exp(const double a[6], double T12[12]) { se3_t T; se3_exp(a, &T); se3_to_mat(&T, T12); }
void orc_se3_left_update(const double a[6], const double T12[12], double out12[12]) {
    se3_t E, T, R;
    se3_exp(a, &E);
    se3_from_mat(T12, &T);
    se3_mul(&E, &T, &R);
    se3_to_mat(&R, out12);
}
void orc_huber(double delta, double e2, double rho[3]) { huber(delta, e2, rho); }
void orc_lu_inverse3(const double A[9], double Ainv[9]) { lu_inverse3(A, Ainv); }
void orc_ldlt_solve(const double *A, int n, const double *b, double *x) {
    double *M = (double *)malloc(sizeof(double) * (size_t)n * (size_t)n);
    memcpy(M, A, sizeof(double) * (size_t)n * (size_t)n);
    ldlt_solve(M, n, b, x);
    free(M);
}
int orc_pcg_solve(const double *A, int n, const double *b, double *x, double tol, int max_iters) {
    return pcg_solve(A, n, b, x, tol, max_iters);
}
/* residual / Jacobians / robust weight of one edge, for finite-difference tests */
void orc_edge_eval(const double T12[12], const double X[3], const double uv[2], const double K[4],
                   const double ext12[12], double huber_delta, double r[2], double Jp[12], double Jl[6],
                   double W[4], double *drho, double *rchi2) {
    prob_t pb;
    memset(&pb, 0, sizeof(pb));
    pb.P = 1; pb.L = 1; pb.O = 1;
    double pose[12], lm[3];
    memcpy(pose, T12, sizeof(pose));
    memcpy(lm, X, sizeof(lm));
    uint32_t z = 0;
    pb.pose = pose; pb.lm = lm; pb.op = &z; pb.ol = &z; pb.uv = uv;
    memcpy(pb.K, K, sizeof(pb.K));
    se3_t ext;
    se3_from_mat(ext12, &ext);
    pb.ext = &ext;
    pb.opt.huber_delta = huber_delta;
    edge_residual(&pb, 0, r);
    edge_jacobians(&pb, 0, Jp, Jl);
    robust_info(&pb, r, W, drho);
    *rchi2 = robust_chi2(&pb, r);
}

/* ============================ frontend pose-only ============================
 * Frontend::EstimateCurrentPose (src/frontend_lego.cpp:157-250): one VertexPose, one
 * EdgeProjectionPoseOnly per tracked feature with a map point (include/legoslam/lego_types.h:116-180),
 * Huber(5.991); four rounds, each restarting from the frame's pose and running
 * problem.solve(10); after each round the outlier flags are refreshed (:205-226) and after the
 * third round the edges lose their cost function (:223-225, so round four is plain least
 * squares).  The flags never remove an edge from the problem (setLevel is commented out, :219,
 * :222).  The Problem is SLAM mode with no landmark vertex: n = 6, the Schur complement is H_pp
 * itself (problem.cpp:380-430 with marg_size 0), and the LM loop is problem.cpp:156-230.
 * Sequential per-edge sums (edge order), LDLT as the backend path.
 */

/* EdgeProjectionPoseOnly::computeResidual (lego_types.h:128-143): K (T X), pi, z - pi */
static void po_residual(const se3_t *T, const double *X, const double *uv, const double *K, double r[2]) {
    double Pc[3];
    se3_apply(T, X, Pc);
    double p0 = K[0] * Pc[0] + 0.0 * Pc[1] + K[2] * Pc[2];
    double p1 = 0.0 * Pc[0] + K[1] * Pc[1] + K[3] * Pc[2];
    double p2 = 0.0 * Pc[0] + 0.0 * Pc[1] + 1.0 * Pc[2];
    double den = p2 + 1e-18;
    p0 /= den; p1 /= den;
    r[0] = uv[0] - p0;
    r[1] = uv[1] - p1;
}

/* EdgeProjectionPoseOnly::computeJacobians (lego_types.h:145-176): J at pos_cam = T X */
static void po_jacobian(const se3_t *T, const double *X, const double *K, double J[12]) {
    double Pc[3];
    se3_apply(T, X, Pc);
    const double fx = K[0], fy = K[1];
    const double x = Pc[0], y = Pc[1], z = Pc[2];
    const double zi = 1.0 / (z + 1e-18);
    const double zi2 = zi * zi;
    J[0] = -fx * zi;              J[1] = 0.0;               J[2] = fx * x * zi2;
    J[3] = fx * x * y * zi2;      J[4] = -fx - fx * x * x * zi2; J[5] = fx * y * zi;
    J[6] = 0.0;                   J[7] = -fy * zi;          J[8] = fy * y * zi2;
    J[9] = fy + fy * y * y * zi2; J[10] = -fy * x * y * zi2; J[11] = -fy * x * zi;
}

typedef struct {
    int32_t O;
    const double *X, *uv;
    double K[4];
    double delta;            /* Huber delta of the edges' cost function, <= 0: none */
    orc_options opt;
    double pose[12], pose_bak[12];
    double *res;             /* O x 2: residual_ as last computed */
    double H[36], b[6], dx[6];
    double chi, lambda, ni;
} po_t;

static double po_rchi2(const po_t *p, const double r[2]) {
    double e2 = r[0] * r[0] + r[1] * r[1];
    if (p->delta > 0) { double rho[3]; huber(p->delta, e2, rho); return rho[0]; }
    return e2;
}

/* buildHessian (problem.cpp:273-358) for the single pose vertex */
static void po_build(po_t *p) {
    se3_t T;
    se3_from_mat(p->pose, &T);
    memset(p->H, 0, sizeof(p->H));
    memset(p->b, 0, sizeof(p->b));
    for (int32_t e = 0; e < p->O; ++e) {
        double r[2], J[12], W[4], drho, Hpp[36];
        po_residual(&T, p->X + 3 * (size_t)e, p->uv + 2 * (size_t)e, p->K, r);
        p->res[2 * e] = r[0]; p->res[2 * e + 1] = r[1];
        po_jacobian(&T, p->X + 3 * (size_t)e, p->K, J);
        if (p->delta > 0) {
            double e2 = r[0] * r[0] + r[1] * r[1], rho[3];
            huber(p->delta, e2, rho);
            W[0] = rho[1]; W[1] = 0.0; W[2] = 0.0; W[3] = rho[1];
            if (rho[1] + 2 * rho[2] * e2 > 0.0) {
                double s = 2 * rho[2];
                W[0] += s * r[0] * r[0]; W[1] += s * r[0] * r[1];
                W[2] += s * r[1] * r[0]; W[3] += s * r[1] * r[1];
            }
            drho = rho[1];
        } else {
            W[0] = 1.0; W[1] = 0.0; W[2] = 0.0; W[3] = 1.0;
            drho = 1.0;
        }
        jtwj(J, 6, W, J, 6, Hpp);
        for (int i = 0; i < 36; ++i) p->H[i] += Hpp[i];
        for (int a = 0; a < 6; ++a) p->b[a] -= (drho * J[a]) * r[0] + (drho * J[6 + a]) * r[1];
    }
    memset(p->dx, 0, sizeof(p->dx));
}

static double po_sum_rchi2(po_t *p, int recompute) {
    se3_t T;
    se3_from_mat(p->pose, &T);
    double s = 0.0;
    for (int32_t e = 0; e < p->O; ++e) {
        if (recompute) po_residual(&T, p->X + 3 * (size_t)e, p->uv + 2 * (size_t)e, p->K, p->res + 2 * e);
        s += po_rchi2(p, p->res + 2 * e);
    }
    return s;
}

/* Problem::solve(max_iters) (problem.cpp:156-230) on the pose-only problem; returns iterations */
static int po_solve(po_t *p, int *trials_out) {
    int trials = 0;
    po_build(p);
    p->ni = 2.0;
    p->chi = 0.5 * po_sum_rchi2(p, 0);
    if (p->opt.strategy == 0) {
        double m = 0.0;
        for (int i = 0; i < 6; ++i) m = fmax(fabs(p->H[7 * i]), m);
        p->lambda = p->opt.lambda_init >= 0 ? p->opt.lambda_init : p->opt.tau * fmin(p->opt.lambda_cap, m);
    } else {
        p->lambda = 1e-5;
    }
    int stop = 0, iter = 0;
    double last_chi = 1e20;
    while (!stop && iter < p->opt.max_iters) {
        int ok = 0, false_cnt = 0;
        while (!ok && false_cnt < p->opt.max_trials) {
            double S[36];
            memcpy(S, p->H, sizeof(S));
            for (int i = 0; i < 6; ++i) {
                if (p->opt.strategy == 0) S[7 * i] += p->lambda;
                else S[7 * i] += p->lambda * S[7 * i];
            }
            ldlt_solve(S, 6, p->b, p->dx);
            memcpy(p->pose_bak, p->pose, sizeof(p->pose));
            {
                double u[6];
                int bad = 0;
                for (int a = 0; a < 6; ++a) if (isnan(p->dx[a]) || isinf(p->dx[a])) bad = 1;
                for (int a = 0; a < 6; ++a) u[a] = bad ? 0.0 : p->dx[a];
                se3_t E, T, R;
                se3_exp(u, &E);
                se3_from_mat(p->pose, &T);
                se3_mul(&E, &T, &R);
                se3_to_mat(&R, p->pose);
            }
            double temp_chi = 0.5 * po_sum_rchi2(p, 1);
            double scale = 0.0;
            for (int i = 0; i < 6; ++i) {
                if (p->opt.strategy == 0) scale += p->dx[i] * (p->lambda * p->dx[i] + p->b[i]);
                else scale += p->dx[i] * (p->lambda * p->H[7 * i] * p->dx[i] + p->b[i]);
            }
            scale = 0.5 * scale;
            scale += 1e-10;
            double rho = (p->chi - temp_chi) / scale;
            ok = rho > 0 && isfinite(temp_chi);
            if (p->opt.strategy == 0) {
                if (ok) {
                    double alpha = 1.0 - pow((2 * rho - 1), 3);
                    alpha = fmin(alpha, 2.0 / 3.0);
                    p->lambda *= fmax(1.0 / 3.0, alpha);
                    p->ni = 2;
                    p->chi = temp_chi;
                } else {
                    p->lambda *= p->ni;
                    p->ni *= 2;
                }
            } else {
                if (ok) { p->lambda = fmax(p->lambda / 9.0, 1e-7); p->chi = temp_chi; }
                else p->lambda = fmin(p->lambda * 11.0, 1e7);
            }
            trials++;
            if (ok) po_build(p);
            else { false_cnt++; memcpy(p->pose, p->pose_bak, sizeof(p->pose)); }
        }
        ++iter;
        if (last_chi - p->chi < p->opt.stop_dchi2) stop = 1;
        last_chi = p->chi;
    }
    if (trials_out) *trials_out += trials;
    return iter;
}

/*
 * orc_estimate_pose — Frontend::EstimateCurrentPose for n_frames independent frames (CSR over
 * observations: frame f owns obs [obs_ptr[f], obs_ptr[f+1])).  pose_in/pose_out [n_frames][12];
 * pts [O][3] map-point positions, uv [O][2]; is_outlier: in = the features' flags on entry
 * (NULL: all false), out = flags after the fourth round.  rchi2_out [O] (optional): each edge's
 * robust chi2 as the last round's classification saw it.  iters_out/trials_out [n_frames]
 * (optional): summed over the four rounds.  Returns 0, or 2 for bad arguments.
 */
int orc_estimate_pose(int32_t n_frames, const int64_t *obs_ptr, const double *pose_in, const double *pts,
                      const double *uv, const double *K, const orc_options *opt, const uint8_t *is_outlier_in,
                      double *pose_out, uint8_t *is_outlier_out, double *rchi2_out, int32_t *iters_out,
                      int32_t *trials_out) {
    if (n_frames < 0 || !obs_ptr || !pose_in || !pose_out || !K || !opt) return 2;
    for (int32_t f = 0; f < n_frames; ++f) {
        const int64_t o0 = obs_ptr[f], O = obs_ptr[f + 1] - o0;
        if (O < 0) return 2;
        po_t p;
        memset(&p, 0, sizeof(p));
        p.O = (int32_t)O;
        p.X = pts + 3 * o0;
        p.uv = uv + 2 * o0;
        memcpy(p.K, K, sizeof(p.K));
        p.opt = *opt;
        p.delta = opt->huber_delta;
        p.res = (double *)calloc(2 * (size_t)(O > 0 ? O : 1), sizeof(double));
        uint8_t *flag = is_outlier_out + o0;
        for (int64_t e = 0; e < O; ++e) flag[e] = is_outlier_in ? is_outlier_in[o0 + e] : 0;
        int its = 0, trials = 0;
        memcpy(p.pose, pose_in + 12 * (size_t)f, sizeof(p.pose));
        for (int round = 0; round < 4; ++round) {
            memcpy(p.pose, pose_in + 12 * (size_t)f, sizeof(p.pose));   /* setEstimate(Pose()) :201 */
            if (O > 0) its += po_solve(&p, &trials);                   /* solve(10): false on no edge */
            se3_t T;
            se3_from_mat(p.pose, &T);
            for (int64_t e = 0; e < O; ++e) {
                if (flag[e]) po_residual(&T, p.X + 3 * e, p.uv + 2 * e, p.K, p.res + 2 * e);   /* :208-210 */
                const double rc = po_rchi2(&p, p.res + 2 * e);
                flag[e] = rc > 5.991;                                   /* chi2_th :171, :211-217 */
                if (rchi2_out) rchi2_out[o0 + e] = rc;
            }
            if (round == 2) p.delta = 0.0;                              /* setCostFunction(nullptr) :223-225 */
        }
        memcpy(pose_out + 12 * (size_t)f, p.pose, sizeof(p.pose));
        if (iters_out) iters_out[f] = its;
        if (trials_out) trials_out[f] = trials;
        free(p.res);
    }
    return 0;
}

/*
 * vo_oracle.c -- CPU ORACLE (test infrastructure; see vo_oracle.h header comment).
 *
 * Plain C restatement of the reference per-frame path.  Every function cites the
 * reference file:line it follows.  Compile with -O2 -ffp-contract=off: all f32/f64
 * expressions are evaluated left to right with one rounding per operation, which is
 * the arithmetic contract the HIP kernels reproduce bit for bit.
 */
#include "vo_oracle.h"
#include "../include/vo_freak_tables.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* Per-stage CPU time of the trajectory loop, the reference's stage timers (VisualOdometry.cpp:85-178:
 * "Feature extraction", "Descriptor matching", "RANSAC", "Pose estimation" around the calls, with
 * get_current_time_fenced, corner_detection_parallel_GPU.h:15-22), extraction split further into its
 * steps (feature_extraction_parallel_GPU.cpp:200-294).  Process-wide (the bench's CPU leg runs one
 * process per core); voo_stage_times reads and voo_stage_reset clears them. */
static double g_stage_s[VOO_NSTAGES];
static int64_t g_stage_n[VOO_NSTAGES];
static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
#define STAGE(k, stmt) do { double _t0 = now_s(); stmt; g_stage_s[k] += now_s() - _t0; g_stage_n[k] += 1; } while (0)
void voo_stage_reset(void) { memset(g_stage_s, 0, sizeof(g_stage_s)); memset(g_stage_n, 0, sizeof(g_stage_n)); }
void voo_stage_times(double* seconds, int64_t* calls)
{
    for (int k = 0; k < VOO_NSTAGES; ++k) { seconds[k] = g_stage_s[k]; calls[k] = g_stage_n[k]; }
}

/* ========================================================================== */
/* deterministic math                                                          */
/* ========================================================================== */

/* atan(i/8) split hi+lo, i = 0..8 (computed with mpmath, 50 digits). */
static const double ATAN_TAB_HI[9] = {
    0.0, 0.12435499454676144, 0.24497866312686414, 0.35877067027057225,
    0.4636476090008061, 0.5585993153435624, 0.6435011087932844,
    0.7188299996216245, 0.7853981633974483};
static const double ATAN_TAB_LO[9] = {
    0.0, -3.1253241424539383e-18, 1.0698755618734451e-17, -2.4623815582638635e-17,
    2.2698777452961687e-17, -5.4556305485916264e-18, 1.5834785051444286e-17,
    -2.1478388444456983e-17, 3.061616997868383e-17};
static const double PI_HI = 3.141592653589793, PI_LO = 1.2246467991473532e-16;
static const double PIO2_HI = 1.5707963267948966, PIO2_LO = 6.123233995736766e-17;
static const double PIO2_1 = 1.570796325802803, PIO2_2 = 9.920935791635221e-10,
                    PIO2_3 = 5.170182981794105e-19;
static const double TWO_OVER_PI = 0.6366197723675814;

/* atan(r), 0 <= r <= 1: r = c + d with c = i/8 nearest, z = (r - c)/(1 + r c),
 * |z| <= 1/16, atan(z) by its odd Taylor series to z^17. */
static double det_atan01(double r)
{
    int i = (int)(r * 8.0 + 0.5);
    double c = (double)i * 0.125;
    double z = (r - c) / (1.0 + r * c);
    double z2 = z * z;
    double p = 1.0 / 17.0;
    p = p * z2 - 1.0 / 15.0;
    p = p * z2 + 1.0 / 13.0;
    p = p * z2 - 1.0 / 11.0;
    p = p * z2 + 1.0 / 9.0;
    p = p * z2 - 1.0 / 7.0;
    p = p * z2 + 1.0 / 5.0;
    p = p * z2 - 1.0 / 3.0;
    double az = z + z * (z2 * p);
    return ATAN_TAB_HI[i] + (az + ATAN_TAB_LO[i]);
}

/* atan2 with C99 quadrant / signed-zero semantics for finite inputs (no NaN). */
double voo_det_atan2(double y, double x)
{
    double ax = fabs(x), ay = fabs(y);
    double t;
    if (ay == 0.0 && ax == 0.0) {
        t = signbit(x) ? PI_HI : 0.0;
    } else if (ay > ax) {
        double b = det_atan01(ax / ay);
        t = signbit(x) ? (PIO2_HI + b) + PIO2_LO : (PIO2_HI - b) + PIO2_LO;
    } else {
        double b = det_atan01(ay / ax);
        t = signbit(x) ? (PI_HI - b) + PI_LO : b;
    }
    if (signbit(y)) t = -t;
    return t;
}

/* sin/cos: Cody-Waite reduction by pi/2 (3-part constant), Taylor polynomials on
 * |r| <= pi/4 (+eps).  Inputs on the path are f32 angles in [-pi, pi]. */
static void det_sincos(double x, double* s_out, double* c_out)
{
    double kf = floor(x * TWO_OVER_PI + 0.5);
    int k = (int)kf;
    double r = ((x - kf * PIO2_1) - kf * PIO2_2) - kf * PIO2_3;
    double r2 = r * r;
    double ps = -1.0 / 355687428096000.0;             /* -1/17! */
    ps = ps * r2 + 1.0 / 1307674368000.0;            /* 1/15!  */
    ps = ps * r2 - 1.0 / 6227020800.0;               /* -1/13! */
    ps = ps * r2 + 1.0 / 39916800.0;                 /* 1/11!  */
    ps = ps * r2 - 1.0 / 362880.0;                   /* -1/9!  */
    ps = ps * r2 + 1.0 / 5040.0;                     /* 1/7!   */
    ps = ps * r2 - 1.0 / 120.0;                      /* -1/5!  */
    ps = ps * r2 + 1.0 / 6.0;                        /* 1/3!   */
    double sr = r - r * (r2 * ps);
    double pc = 1.0 / 6402373705728000.0;             /* 1/18!  */
    pc = pc * r2 - 1.0 / 20922789888000.0;           /* -1/16! */
    pc = pc * r2 + 1.0 / 87178291200.0;              /* 1/14!  */
    pc = pc * r2 - 1.0 / 479001600.0;                /* -1/12! */
    pc = pc * r2 + 1.0 / 3628800.0;                  /* 1/10!  */
    pc = pc * r2 - 1.0 / 40320.0;                    /* -1/8!  */
    pc = pc * r2 + 1.0 / 720.0;                      /* 1/6!   */
    pc = pc * r2 - 1.0 / 24.0;                       /* -1/4!  */
    pc = pc * r2 + 0.5;                              /* 1/2!   */
    double cr = 1.0 - r2 * pc;
    switch (k & 3) {
    case 0: *s_out = sr;  *c_out = cr;  break;
    case 1: *s_out = cr;  *c_out = -sr; break;
    case 2: *s_out = -sr; *c_out = -cr; break;
    default: *s_out = -cr; *c_out = sr; break;
    }
}
double voo_det_sin(double x) { double s, c; det_sincos(x, &s, &c); return s; }
double voo_det_cos(double x) { double s, c; det_sincos(x, &s, &c); return c; }

uint64_t voo_mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

uint64_t voo_frame_seed(uint64_t seed, int64_t frame)
{
    return voo_mix64(seed + 0x632BE59BD9B4E019ULL * (uint64_t)(frame + 1));
}

/* Hypothesis k's minimal sample: 8 distinct indices of [0, m), ascending.
 * Replaces std::sample(data, 8, std::mt19937(std::random_device{}())) (ransac.cpp:137,142),
 * which is irreproducible by construction; same distribution (uniform 8-subset, kept
 * in data order like libstdc++'s selection sampling).  Floyd's algorithm. */
void voo_sample8(uint64_t seed, int k, int m, int32_t out[8])
{
    uint64_t st = voo_mix64(seed ^ (0x9E3779B97F4A7C15ULL * (uint64_t)(k + 1)));
    int cnt = 0;
    for (int j = m - 8; j < m; ++j) {
        st += 0x9E3779B97F4A7C15ULL;
        uint64_t r = voo_mix64(st);
        uint32_t t = (uint32_t)(((unsigned __int128)r * (uint64_t)(j + 1)) >> 64);
        int present = 0;
        for (int i = 0; i < cnt; ++i) present |= (out[i] == (int32_t)t);
        out[cnt++] = present ? j : (int32_t)t;
    }
    for (int i = 1; i < 8; ++i) {
        int32_t v = out[i];
        int j = i - 1;
        while (j >= 0 && out[j] > v) { out[j + 1] = out[j]; --j; }
        out[j + 1] = v;
    }
}

/* x86 cvttsd2si: truncation; NaN / out of range -> INT_MIN (the reference's
 * double->int assignment at ransac.cpp:131,186 is UB in C++ and compiles to this). */
static int to_int_x86(double q)
{
    if (!(q > -2147483649.0 && q < 2147483648.0)) return INT_MIN;
    return (int)q;
}

int voo_ransac_maxit_initial(double prob)
{
    double outlierRatio = 0.5;
    return to_int_x86(log(1.0 - prob) / log(1.0 - pow(1.0 - outlierRatio, 8.0)));
}

/* ransac.cpp:179-190: recomputed on each strictly better inlier count. Returns
 * -1 when denom == 0 (no update). */
int voo_ransac_maxit_update(int best, int n, double prob)
{
    double outlierRatio = 1.0 - (double)best / (double)n;
    double denom = log(1.0 - pow(1.0 - outlierRatio, 8.0));
    if (denom == 0.0) return -1;
    int it = to_int_x86(log(1.0 - prob) / denom);
    if (it < 100) it = 100;
    if (it > 2000) it = 2000;
    return it;
}

/* ========================================================================== */
/* small dense linear algebra (f64, fixed operation order)                      */
/* ========================================================================== */


static void mm3(const double* A, const double* B, double* C);
static void mtm3(const double* A, const double* B, double* C);

/* Least-squares null vector of the refit's design matrix: the smallest eigenvector of the
 * 9x9 PSD S = A^T A (Eigen::JacobiSVD V.col(8), ransac.cpp:77-78).
 *   1. Cholesky S = L L^T with a pivot floor of 1e-15 * max diag (an exactly singular S --
 *      e.g. 8 inliers -- has its null vector as the dominant direction of S^-1);
 *   2. W = S^-1 = L^-T L^-1 from the column-wise inverse of L, squared six times to W^64, each
 *      power first scaled by the power of two that brings its largest diagonal entry into
 *      [0.5, 1) (exact; eigenvectors unchanged);
 *   3. power iteration x <- W64 x / |W64 x| (sign kept towards x) from the warm start x0 until
 *      the unit iterate moves by <= 4e-16 (at most 32 steps; one step = 64 inverse iterations);
 *   4. no convergence: keep x if its Rayleigh quotient certifies it in S's numerical null space,
 *      else cyclic Jacobi on S (voo_dbg_nullvec_status says which).
 * Every entry's sum runs in ascending index order; k_refit computes the same entries lane-
 * parallel in that order, so the two agree bit for bit. */
int voo_dbg_nullvec_iters;
#define NV_CONVERGED 0      /* the power iterate moved by <= 4e-16 */
#define NV_CERTIFIED 1      /* 32 steps, iterate's Rayleigh quotient at the Cholesky floor: in the null space */
#define NV_JACOBI 2         /* 32 steps, above the floor: cyclic Jacobi fallback */
int voo_dbg_nullvec_status;
double voo_dbg_refit_f[9];
static double* voo_dbg_capture_normal;   /* voo_refit_normal: where the refit copies A^T A */   /* test hook: the last refit's normalized null vector (before denormalization) */
/* power of two r with max_i W_ii * r in [0.5, 1): W is symmetric PSD, so |W_ij| <= max_i W_ii,
 * and scaling by r is exact (the squarings only need it to keep clear of overflow) */
static double pow2_scale9(const double* W)
{
    double m = 0.0;
    for (int i = 0; i < 9; ++i) if (W[i * 9 + i] > m) m = W[i * 9 + i];
    int e;
    (void)frexp(m, &e);
    return ldexp(1.0, -e);
}
static void sym_square9(const double* A, double r, double* B)   /* B = (rA)(rA), A symmetric, sums k-ascending */
{
    for (int i = 0; i < 9; ++i)
        for (int j = i; j < 9; ++j) {
            double v = 0.0;
            for (int k = 0; k < 9; ++k) v = v + (A[i * 9 + k] * r) * (A[k * 9 + j] * r);
            B[i * 9 + j] = v; B[j * 9 + i] = v;
        }
}
/* x^T S x, sums in ascending index order (x unit) */
static double nv_rayleigh9(const double* S, const double* x)
{
    double rq = 0.0;
    for (int i = 0; i < 9; ++i) {
        double si = 0.0;
        for (int j = 0; j < 9; ++j) si = si + S[i * 9 + j] * x[j];
        rq = rq + x[i] * si;
    }
    return rq;
}

/* Smallest eigenvector of the 9x9 symmetric S by cyclic Jacobi (the classic rotation
 * t = sgn(th) / (|th| + sqrt(th^2 + 1)), th = (a_qq - a_pp) / (2 a_pq); pairs p < q in row order;
 * an off-diagonal entry at or below 1e-18 of the diagonal's magnitude is set to zero; at most 64
 * sweeps, ending at the first sweep that finds every off-diagonal entry zero).  The eigenvector of
 * the first smallest diagonal entry, signed towards x0 (the warm start). */
static void jacobi_min_eigvec9(const double* S, const double* x0, double* f)
{
    double a[81], v[81];
    for (int i = 0; i < 81; ++i) { a[i] = S[i]; v[i] = (i % 10 == 0) ? 1.0 : 0.0; }
    for (int sweep = 0; sweep < 64; ++sweep) {
        int rot = 0;
        for (int p = 0; p < 8; ++p)
            for (int q = p + 1; q < 9; ++q) {
                double apq = a[p * 9 + q];
                if (apq == 0.0) continue;
                if (fabs(apq) <= 1e-18 * (fabs(a[p * 9 + p]) + fabs(a[q * 9 + q]))) {
                    a[p * 9 + q] = 0.0; a[q * 9 + p] = 0.0;
                    continue;
                }
                ++rot;
                double th = (a[q * 9 + q] - a[p * 9 + p]) / (2.0 * apq);
                double t = 1.0 / (fabs(th) + sqrt(th * th + 1.0));
                if (th < 0.0) t = -t;
                double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 9; ++k) {            /* columns p, q */
                    double akp = a[k * 9 + p], akq = a[k * 9 + q];
                    a[k * 9 + p] = c * akp - s * akq;
                    a[k * 9 + q] = s * akp + c * akq;
                }
                for (int k = 0; k < 9; ++k) {            /* rows p, q */
                    double apk = a[p * 9 + k], aqk = a[q * 9 + k];
                    a[p * 9 + k] = c * apk - s * aqk;
                    a[q * 9 + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 9; ++k) {
                    double vkp = v[k * 9 + p], vkq = v[k * 9 + q];
                    v[k * 9 + p] = c * vkp - s * vkq;
                    v[k * 9 + q] = s * vkp + c * vkq;
                }
            }
        if (!rot) break;
    }
    int k = 0;
    for (int i = 1; i < 9; ++i) if (a[i * 9 + i] < a[k * 9 + k]) k = i;
    double dot = 0.0;
    for (int i = 0; i < 9; ++i) dot = dot + v[i * 9 + k] * x0[i];
    double sg = dot < 0.0 ? -1.0 : 1.0;
    for (int i = 0; i < 9; ++i) f[i] = v[i * 9 + k] * sg;
}

static void ls_nullvec9(const double* S, const double* x0, double* f)
{
    double L[81], invd[9], Li[81], W[81], W2[81];
    double mx = 0.0;
    for (int i = 0; i < 9; ++i)
        if (S[i * 9 + i] > mx) mx = S[i * 9 + i];
    double fl = 1e-15 * mx;
    if (!(fl > 0.0)) fl = 1e-300;
    for (int i = 0; i < 81; ++i) { L[i] = 0.0; Li[i] = 0.0; }
    for (int j = 0; j < 9; ++j) {
        double sj = S[j * 9 + j];
        for (int k = 0; k < j; ++k) sj = sj - L[j * 9 + k] * L[j * 9 + k];
        if (!(sj > fl)) sj = fl;
        double dj = sqrt(sj);
        L[j * 9 + j] = dj;
        invd[j] = 1.0 / dj;
        for (int i = j + 1; i < 9; ++i) {
            double v = S[i * 9 + j];
            for (int k = 0; k < j; ++k) v = v - L[i * 9 + k] * L[j * 9 + k];
            L[i * 9 + j] = v * invd[j];
        }
    }
    for (int c = 0; c < 9; ++c) {             /* column c of L^-1 by forward substitution */
        Li[c * 9 + c] = invd[c];
        for (int i = c + 1; i < 9; ++i) {
            double v = 0.0;
            for (int k = c; k < i; ++k) v = v + L[i * 9 + k] * Li[k * 9 + c];
            Li[i * 9 + c] = -(v * invd[i]);
        }
    }
    for (int i = 0; i < 9; ++i)               /* W = L^-T L^-1: W_ij = sum_{k>=j} Li_ki Li_kj, i <= j */
        for (int j = i; j < 9; ++j) {
            double v = 0.0;
            for (int k = j; k < 9; ++k) v = v + Li[k * 9 + i] * Li[k * 9 + j];
            W[i * 9 + j] = v; W[j * 9 + i] = v;
        }
    for (int q = 0; q < 3; ++q) {              /* W <- W^64 */
        sym_square9(W, pow2_scale9(W), W2);
        sym_square9(W2, pow2_scale9(W2), W);
    }
    double x[9];
    double n0 = 0.0;
    for (int i = 0; i < 9; ++i) n0 = n0 + x0[i] * x0[i];
    n0 = sqrt(n0);
    if (n0 > 0.0 && n0 < 1e300) { for (int i = 0; i < 9; ++i) x[i] = x0[i] / n0; }
    else { for (int i = 0; i < 9; ++i) x[i] = 1.0 / 3.0; }
    int it = 0, conv = 0;
    for (; it < 32; ++it) {
        double z[9];
        for (int i = 0; i < 9; ++i) {
            double v = 0.0;
            for (int j = 0; j < 9; ++j) v = v + W[i * 9 + j] * x[j];
            z[i] = v;
        }
        double nn = 0.0, dot = 0.0;
        for (int i = 0; i < 9; ++i) { nn = nn + z[i] * z[i]; dot = dot + z[i] * x[i]; }
        nn = sqrt(nn);
        double r = (dot < 0.0 ? -1.0 : 1.0) / nn;
        double diff = 0.0;
        for (int i = 0; i < 9; ++i) {
            double xn = z[i] * r;
            double dd = fabs(xn - x[i]);
            if (dd > diff) diff = dd;
            x[i] = xn;
        }
        if (diff <= 4e-16) { ++it; conv = 1; break; }
    }
    voo_dbg_nullvec_iters = it;
    voo_dbg_nullvec_status = NV_CONVERGED;
    if (!conv) {
        /* No convergence in 32 steps (2048 inverse iterations): the two smallest eigenvalues of S
         * are within a factor ~1 - 1e-5.  If the iterate's Rayleigh quotient is at the Cholesky floor,
         * it lies in S's numerical null space (several directions below the floor: a degenerate set,
         * where any null vector is as good as JacobiSVD's pick) and is kept; otherwise the smallest
         * eigenvector comes from cyclic Jacobi on S. */
        if (nv_rayleigh9(S, x) <= 64.0 * fl) voo_dbg_nullvec_status = NV_CERTIFIED;
        else { jacobi_min_eigvec9(S, x0, x); voo_dbg_nullvec_status = NV_JACOBI; }
    }
    for (int i = 0; i < 9; ++i) f[i] = x[i];
}

/* test hook: ls_nullvec9 on a given S; returns the status (NV_*) */
int voo_ls_nullvec9(const double* S, const double* x0, double* f)
{
    ls_nullvec9(S, x0, f);
    return voo_dbg_nullvec_status;
}

/* warm start for ls_nullvec9: the best hypothesis' F mapped into the refit's normalized
 * frame, f0 = T2^-T F T1^-1 (inverse of the quirk-6 denormalization F = T2^T f T1). */
static void warm_start(const double* Fb, double s1, double mx1, double my1, double s2, double mx2, double my2,
                       double* f0)
{
    double T1i[9] = {1.0 / s1, 0.0, mx1, 0.0, 1.0 / s1, my1, 0.0, 0.0, 1.0};
    double T2i[9] = {1.0 / s2, 0.0, mx2, 0.0, 1.0 / s2, my2, 0.0, 0.0, 1.0};
    double G[9];
    mtm3(T2i, Fb, G);
    mm3(G, T1i, f0);
}


/* C = A(3x3) * B(3x3), sums in k order. */
static void mm3(const double* A, const double* B, double* C)
{
    double T[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            T[i * 3 + j] = (A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j]) + A[i * 3 + 2] * B[2 * 3 + j];
    memcpy(C, T, sizeof(T));
}
static void mtm3(const double* A, const double* B, double* C) /* C = A^T B */
{
    double T[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            T[i * 3 + j] = (A[0 * 3 + i] * B[0 * 3 + j] + A[1 * 3 + i] * B[1 * 3 + j]) + A[2 * 3 + i] * B[2 * 3 + j];
    memcpy(C, T, sizeof(T));
}
static double det3(const double* M)
{
    return (M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6])) +
           M[2] * (M[3] * M[7] - M[4] * M[6]);
}

/* Unit eigenvector of the smallest eigenvalue of a 3x3 symmetric PSD S: the dominant
 * eigenvector of adj(S) (eigenvalues l2 l3, l1 l3, l1 l2), squared four times (each power
 * first scaled by the power of two bringing its largest diagonal entry into [0.5, 1)),
 * started from its largest-diagonal column and power-iterated until the unit iterate moves
 * by <= 4e-16 (at most 32 steps).  adj(S) = 0 (rank <= 1) gives e3. */
static void min_eigvec3(const double* S, double* v)
{
    double B[9], B2[9];
    B[0] = S[4] * S[8] - S[5] * S[7];
    B[4] = S[0] * S[8] - S[2] * S[6];
    B[8] = S[0] * S[4] - S[1] * S[3];
    B[1] = -(S[3] * S[8] - S[5] * S[6]); B[3] = B[1];
    B[2] = S[3] * S[7] - S[4] * S[6];    B[6] = B[2];
    B[5] = -(S[0] * S[7] - S[1] * S[6]); B[7] = B[5];
    int k = 0;
    for (int i = 1; i < 3; ++i) if (B[i * 3 + i] > B[k * 3 + k]) k = i;
    if (!(B[k * 3 + k] > 0.0)) { v[0] = 0.0; v[1] = 0.0; v[2] = 1.0; return; }
    for (int q = 0; q < 4; ++q) {
        double m = 0.0;
        for (int i = 0; i < 3; ++i) if (B[i * 3 + i] > m) m = B[i * 3 + i];
        int e;
        (void)frexp(m, &e);
        double r = ldexp(1.0, -e);
        for (int i = 0; i < 3; ++i)
            for (int j = i; j < 3; ++j) {
                double x = ((B[i * 3 + 0] * r) * (B[0 * 3 + j] * r) + (B[i * 3 + 1] * r) * (B[1 * 3 + j] * r)) +
                           (B[i * 3 + 2] * r) * (B[2 * 3 + j] * r);
                B2[i * 3 + j] = x; B2[j * 3 + i] = x;
            }
        memcpy(B, B2, sizeof(B2));
    }
    k = 0;
    for (int i = 1; i < 3; ++i) if (B[i * 3 + i] > B[k * 3 + k]) k = i;
    double nn = (B[0 * 3 + k] * B[0 * 3 + k] + B[1 * 3 + k] * B[1 * 3 + k]) + B[2 * 3 + k] * B[2 * 3 + k];
    double rn = 1.0 / sqrt(nn);
    for (int i = 0; i < 3; ++i) v[i] = B[i * 3 + k] * rn;
    for (int it = 0; it < 32; ++it) {
        double z[3];
        for (int i = 0; i < 3; ++i) z[i] = (B[i * 3 + 0] * v[0] + B[i * 3 + 1] * v[1]) + B[i * 3 + 2] * v[2];
        double zz = (z[0] * z[0] + z[1] * z[1]) + z[2] * z[2];
        double dot = (z[0] * v[0] + z[1] * v[1]) + z[2] * v[2];
        double rs = (dot < 0.0 ? -1.0 : 1.0) / sqrt(zz);
        double diff = 0.0;
        for (int i = 0; i < 3; ++i) {
            double xn = z[i] * rs;
            double dd = fabs(xn - v[i]);
            if (dd > diff) diff = dd;
            v[i] = xn;
        }
        if (diff <= 4e-16) break;
    }
}

/* Rank-2 projection F <- U diag(s1,s2,0) V^T == F (I - v3 v3^T)  (ransac.cpp:87-90), v3 the
 * smallest eigenvector of F^T F (min_eigvec3). */
static void rank2(double* F)
{
    double FtF[9], v[3];
    mtm3(F, F, FtF);
    min_eigvec3(FtF, v);
    double v0 = v[0], v1 = v[1], v2 = v[2];
    for (int i = 0; i < 3; ++i) {
        double fv = (F[i * 3 + 0] * v0 + F[i * 3 + 1] * v1) + F[i * 3 + 2] * v2;
        F[i * 3 + 0] = F[i * 3 + 0] - fv * v0;
        F[i * 3 + 1] = F[i * 3 + 1] - fv * v1;
        F[i * 3 + 2] = F[i * 3 + 2] - fv * v2;
    }
}

/* F = T2^T F0 T1 with T = [[s,0,-s mx],[0,s,-s my],[0,0,1]]   (ransac.cpp:85). */
static void denormalize(const double* F0, double s1, double mx1, double my1,
                        double s2, double mx2, double my2, double* F)
{
    double T1[9] = {s1, 0.0, -(s1 * mx1), 0.0, s1, -(s1 * my1), 0.0, 0.0, 1.0};
    double T2[9] = {s2, 0.0, -(s2 * mx2), 0.0, s2, -(s2 * my2), 0.0, 0.0, 1.0};
    double G[9];
    mtm3(T2, F0, G);
    mm3(G, T1, F);
}

/* One design-matrix row (ransac.cpp:72-74) from normalized p1, p2. */
static void design_row(double p1x, double p1y, double p2x, double p2y, double* a)
{
    a[0] = p1x * p2x; a[1] = p1x * p2y; a[2] = p1x;
    a[3] = p1y * p2x; a[4] = p1y * p2y; a[5] = p1y;
    a[6] = p2x; a[7] = p2y; a[8] = 1.0;
}

/* Null vector of the 8x9 design matrix: Gauss-Jordan elimination with complete
 * pivoting (pivot = first max |a| in row-major order over unused rows/cols), then
 * x_free = 1, x_pc = -a[pr][free]/a[pr][pc], unit-normalized.  This is the exact
 * (1-D) null space that Eigen::JacobiSVD's V.col(8) spans (ransac.cpp:77-78). */
static void nullvec_8x9(double M[8][9], double f[9])
{
    int used_r[8] = {0}, used_c[9] = {0}, pr_[8], pc_[8];
    int steps = 0;
    for (int step = 0; step < 8; ++step) {
        double best = 0.0; int br = -1, bc = -1;
        for (int r = 0; r < 8; ++r) {
            if (used_r[r]) continue;
            for (int c = 0; c < 9; ++c) {
                if (used_c[c]) continue;
                double a = fabs(M[r][c]);
                if (a > best) { best = a; br = r; bc = c; }
            }
        }
        if (br < 0) break;
        used_r[br] = 1; used_c[bc] = 1; pr_[step] = br; pc_[step] = bc; steps = step + 1;
        double piv = M[br][bc];
        for (int r = 0; r < 8; ++r) {
            if (r == br) continue;
            double fct = M[r][bc] / piv;
            for (int c = 0; c < 9; ++c) M[r][c] = M[r][c] - fct * M[br][c];
        }
    }
    int fc = 0;
    while (fc < 9 && used_c[fc]) ++fc;
    for (int c = 0; c < 9; ++c) f[c] = 0.0;
    f[fc] = 1.0;
    for (int s = 0; s < steps; ++s) f[pc_[s]] = -(M[pr_[s]][fc] / M[pr_[s]][pc_[s]]);
    double nn = 0.0;
    for (int c = 0; c < 9; ++c) nn = nn + f[c] * f[c];
    nn = sqrt(nn);
    for (int c = 0; c < 9; ++c) f[c] = f[c] / nn;
}

/* Fixed-order parallel sum used by the device refit (128 threads): thread t accumulates
 * elements t, t+128, ... in order; the total sums the 128 partials in thread order as 8
 * sequential chains of 16, combined pairwise.  The oracle reproduces that order so refit
 * outputs compare bit for bit. */
#define VOO_RED_THREADS 128
typedef struct { double v[VOO_RED_THREADS]; } red256;
static double red_finish(red256* r)
{
    double c[8];
    for (int j = 0; j < 8; ++j) {
        c[j] = 0.0;
        for (int t = 0; t < 16; ++t) c[j] = c[j] + r->v[16 * j + t];
    }
    return ((c[0] + c[1]) + (c[2] + c[3])) + ((c[4] + c[5]) + (c[6] + c[7]));
}

/* ========================================================================== */
/* extract                                                                      */
/* ========================================================================== */

static int refl101(int i, int n)
{
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        else i = 2 * n - 2 - i;
    }
    return i;
}

/* cv::GaussianBlur(img, out, Size(7,7), 0) on CV_8U (feature_extraction_parallel_GPU.cpp:200):
 * OpenCV 4 bit-exact fixed-point path, taps {8,28,56,72,56,28,8}/256 (sigma<=0, ksize 7),
 * BORDER_REFLECT_101, out = (sum_a k_a sum_b k_b I + 2^15) >> 16. */
void voo_blur7(const uint8_t* src, size_t stride, int W, int H, uint8_t* dst)
{
    static const int k[7] = {8, 28, 56, 72, 56, 28, 8};
    uint32_t* tmp = (uint32_t*)malloc((size_t)W * H * sizeof(uint32_t));
    for (int y = 0; y < H; ++y) {
        const uint8_t* row = src + (size_t)y * stride;
        for (int x = 0; x < W; ++x) {
            uint32_t h = 0;
            for (int b = 0; b < 7; ++b) h += (uint32_t)k[b] * row[refl101(x + b - 3, W)];
            tmp[(size_t)y * W + x] = h;
        }
    }
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            uint32_t v = 0;
            for (int a = 0; a < 7; ++a) v += (uint32_t)k[a] * tmp[(size_t)refl101(y + a - 3, H) * W + x];
            dst[(size_t)y * W + x] = (uint8_t)((v + 32768u) >> 16);
        }
    }
    free(tmp);
}

/* gradient_convolution, kernels/feature_extraction_kernel_functions.c:43-78.
 * Computed for 1<=i<=H-2, 1<=j<=W-2 (launch corner_detection_parallel_GPU.cpp:69-72); border 0. */
void voo_gradients(const uint8_t* b, int W, int H, float* Jx, float* Jy, float* Jxy)
{
    memset(Jx, 0, sizeof(float) * W * H);
    memset(Jy, 0, sizeof(float) * W * H);
    memset(Jxy, 0, sizeof(float) * W * H);
    for (int i = 1; i <= H - 2; ++i) {
        for (int j = 1; j <= W - 2; ++j) {
            const uint8_t* a = b + (size_t)(i - 1) * W;
            const uint8_t* m = b + (size_t)i * W;
            const uint8_t* c = b + (size_t)(i + 1) * W;
            float sumx[3], sumy[3];
            for (int k = -1; k <= 1; ++k) {
                sumx[k + 1] = (float)a[j + k] - (float)c[j + k];
                sumy[k + 1] = ((float)a[j + k] + 2.0f * (float)m[j + k]) + (float)c[j + k];
            }
            size_t idx = (size_t)i * W + j;
            Jx[idx] = (sumx[0] + 2.0f * sumx[1]) + sumx[2];
            Jy[idx] = sumy[0] - sumy[2];
            Jxy[idx] = sumx[0] - sumx[2];
        }
    }
}

/* shitomasi_response, kernels/feature_extraction_kernel_functions.c:81-120.
 * For 2<=i<=H-3, 2<=j<=W-3 (launch corner_detection_parallel_GPU.cpp:96-99); border 0. */
void voo_response(const uint8_t* b, int W, int H, float thr, float* R)
{
    float* Jx = (float*)malloc(sizeof(float) * W * H);
    float* Jy = (float*)malloc(sizeof(float) * W * H);
    float* Jxy = (float*)malloc(sizeof(float) * W * H);
    voo_gradients(b, W, H, Jx, Jy, Jxy);
    memset(R, 0, sizeof(float) * W * H);
    for (int i = 2; i <= H - 3; ++i) {
        for (int j = 2; j <= W - 3; ++j) {
            float jx2 = 0.0f, jy2 = 0.0f, s = 0.0f;
            for (int m = -2; m <= 2; ++m) {
                for (int n = -2; n <= 2; ++n) {
                    size_t q = (size_t)(i + m) * W + (j + n);
                    float jx = Jx[q], jy = Jy[q], jxy = Jxy[q];
                    s = s + jxy;
                    jx2 = jx2 + jx * jx;
                    jy2 = jy2 + jy * jy;
                }
            }
            float det = (jx2 * jy2) - (s * s);
            float tr = jx2 + jy2;
            float r = (tr / 2.0f) - (0.5f * sqrtf(tr * tr - 4.0f * det));
            R[(size_t)i * W + j] = r > thr ? r : 0.0f;
        }
    }
    free(Jx); free(Jy); free(Jxy);
}

typedef struct { float r; int i, j; } voo_cand;

/* (R, i, j) lexicographic descending: the std::priority_queue<tuple<float,int,int>> pop order. */
static int cand_cmp_desc(const void* pa, const void* pb)
{
    const voo_cand* a = (const voo_cand*)pa;
    const voo_cand* b = (const voo_cand*)pb;
    if (a->r != b->r) return a->r > b->r ? -1 : 1;
    if (a->i != b->i) return a->i > b->i ? -1 : 1;
    if (a->j != b->j) return a->j > b->j ? -1 : 1;
    return 0;
}
static int kp_cmp_raster(const void* pa, const void* pb)
{
    const int32_t* a = (const int32_t*)pa;
    const int32_t* b = (const int32_t*)pb;
    if (a[1] != b[1]) return a[1] < b[1] ? -1 : 1;
    if (a[0] != b[0]) return a[0] < b[0] ? -1 : 1;
    return 0;
}

static int nms_collect(const float* R, int W, int H, int k, int brow, int bcol, voo_cand* out)
{
    int h = k / 2, n = 0;
    for (int i = h; i < H - h; ++i) {
        for (int j = h; j < W - h; ++j) {
            if (!((j >= bcol) && (j <= W - bcol) && (i >= brow) && (i <= H - brow))) continue;
            float cv = R[(size_t)i * W + j];
            int is_max = 1;
            for (int a = i - h; a <= i + h && is_max; ++a)
                for (int b = j - h; b <= j + h; ++b) {
                    if (a == i && b == j) continue;
                    if (R[(size_t)a * W + b] >= cv) { is_max = 0; break; }
                }
            if (is_max) {
                if (out) { out[n].r = cv; out[n].i = i; out[n].j = j; }
                ++n;
            }
        }
    }
    return n;
}

int voo_nms_candidates(const float* R, int W, int H, int k, int brow, int bcol)
{
    return nms_collect(R, W, H, k, brow, bcol, NULL);
}

/* non_maximum_suppression(R, H, W, k, N), corner_detection_parallel_GPU.cpp:146-188, followed by
 * the (row, col) sort of feature_extraction_parallel_GPU.cpp:259-265.  kps_xy: x=col, y=row. */
int voo_nms_topn(const float* R, int W, int H, int k, int N, int brow, int bcol, int32_t* kps_xy)
{
    int nc = nms_collect(R, W, H, k, brow, bcol, NULL);
    voo_cand* c = (voo_cand*)malloc(sizeof(voo_cand) * (nc > 0 ? nc : 1));
    nms_collect(R, W, H, k, brow, bcol, c);
    qsort(c, nc, sizeof(voo_cand), cand_cmp_desc);
    int n = nc < N ? nc : N;
    for (int t = 0; t < n; ++t) { kps_xy[2 * t] = c[t].j; kps_xy[2 * t + 1] = c[t].i; }
    qsort(kps_xy, n, 2 * sizeof(int32_t), kp_cmp_raster);
    free(c);
    return n;
}

/* Orientation sums in the deterministic order of FREAK_Parallel::compute_orientation
 * (feature_extraction_parallel/FREAK_feature_descriptor_parallel.cpp:16-44): pairs (i<j)
 * row-major, f32, O = 0 + sum (I_i - I_j) * d / |d|.  Per-term arithmetic as
 * compute_all_orientations (kernels/feature_extraction_kernel_functions.c:142-160). */
void voo_orientation(const uint8_t* img, int W, int kx, int ky, float* ox, float* oy)
{
    float Ox = 0.0f, Oy = 0.0f;
    for (int p = 0; p < VO_FREAK_NPOINTS; ++p) {
        int px = vo_freak_points[p][0], py = vo_freak_points[p][1];
        float i1 = (float)img[(size_t)(ky + py) * W + (kx + px)];
        for (int q = p + 1; q < VO_FREAK_NPOINTS; ++q) {
            int qx = vo_freak_points[q][0], qy = vo_freak_points[q][1];
            float i2 = (float)img[(size_t)(ky + qy) * W + (kx + qx)];
            float ic = i1 - i2;
            float dx = (float)(px - qx), dy = (float)(py - qy);
            float nrm = sqrtf(dx * dx + dy * dy);
            if (nrm == 0.0f) continue;
            Ox = Ox + (ic * dx) / nrm;
            Oy = Oy + (ic * dy) / nrm;
        }
    }
    *ox = Ox; *oy = Oy;
}

/* FREAK_Parallel_GPU::FREAK_feature_description (FREAK_feature_descriptor_parallel_GPU.cpp:10-210):
 * merge_all_orientations (kernel .c:169-195) + compute_all_descriptors (kernel .c:198-225).
 * Descriptor bit t (test t = 0..511) is stored LSB-first in u64 word t/64 (byte-per-test
 * layout of the reference == unpack of these words).  rot (optional): c, -s, s, c. */
void voo_describe(const uint8_t* img, int W, int H, const int32_t* kps, int n, uint64_t* desc, float* rot)
{
    (void)H;
    for (int k = 0; k < n; ++k) {
        int kx = kps[2 * k], ky = kps[2 * k + 1];
        float Ox, Oy;
        voo_orientation(img, W, kx, ky, &Ox, &Oy);
        float angle = 0.0f;
        if (!(isnan(Ox) || isnan(Oy))) angle = (float)voo_det_atan2((double)Oy, (double)Ox);
        float c = (float)voo_det_cos((double)angle);
        float s = (float)voo_det_sin((double)angle);
        float ms = -1.0f * s;                   /* rotation_matrix[1] */
        if (rot) { rot[4 * k] = c; rot[4 * k + 1] = ms; rot[4 * k + 2] = s; rot[4 * k + 3] = c; }
        /* the 43 sample points after the (non-orthogonal) transform, kernel .c:214-220 */
        uint8_t I[VO_FREAK_NPOINTS];
        for (int p = 0; p < VO_FREAK_NPOINTS; ++p) {
            int px = vo_freak_points[p][0], py = vo_freak_points[p][1];
            int x = (int)(((float)kx + (float)px * c) + (float)py * s);
            int y = (int)(((float)ky + (float)(-1 * px) * ms) + (float)py * c);
            I[p] = img[(size_t)y * W + x];
        }
        uint64_t w[8] = {0};
        int t = 0;
        /* pair index -> (p, q): iterate the pair enumeration once */
        static int pair_p[VO_FREAK_NPAIRS], pair_q[VO_FREAK_NPAIRS], init = 0;
        if (!init) {
            int e = 0;
            for (int p = 0; p < VO_FREAK_NPOINTS; ++p)
                for (int q = p + 1; q < VO_FREAK_NPOINTS; ++q) { pair_p[e] = p; pair_q[e] = q; ++e; }
            init = 1;
        }
        for (t = 0; t < VO_FREAK_NTESTS; ++t) {
            int e = vo_freak_patch[t];
            if (I[pair_p[e]] > I[pair_q[e]]) w[t >> 6] |= 1ULL << (t & 63);
        }
        memcpy(desc + 8 * (size_t)k, w, sizeof(w));
    }
}

int voo_extract(const voo_config* cf, const uint8_t* gray, size_t stride, int32_t* kps, uint64_t* desc,
                uint8_t* blurred_out)
{
    int W = cf->width, H = cf->height;
    uint8_t* bl = (uint8_t*)malloc((size_t)W * H);
    float* R = (float*)malloc(sizeof(float) * W * H);
    int n;
    STAGE(VOO_STAGE_BLUR, voo_blur7(gray, stride, W, H, bl));
    STAGE(VOO_STAGE_RESPONSE, voo_response(bl, W, H, cf->resp_thr, R));
    STAGE(VOO_STAGE_NMS, n = voo_nms_topn(R, W, H, cf->nms_k, cf->max_kpts, cf->border_row, cf->border_col, kps));
    STAGE(VOO_STAGE_DESCRIBE, voo_describe(bl, W, H, kps, n, desc, NULL));
    if (blurred_out) memcpy(blurred_out, bl, (size_t)W * H);
    free(bl); free(R);
    return n;
}

/* ========================================================================== */
/* match                                                                        */
/* ========================================================================== */

static int hamming(const uint64_t* a, const uint64_t* b, int bits)
{
    if (bits == 32) return __builtin_popcountll((a[0] ^ b[0]) & 0xFFFFFFFFULL);
    int d = 0;
    for (int w = 0; w < 8; ++w) d += __builtin_popcountll(a[w] ^ b[w]);
    return d;
}

/* matchCustomBinaryDescriptorsThreadPool (feature_matching_parallel.cpp:49-113): the
 * reference XORs 4 u64 words of the 512-byte 0/1 vector = tests 0..31 (quirk 1);
 * match_bits = 512 gives matching_serial.cpp:42-77 (full length).  Output in ascending i. */
int voo_match(const uint64_t* d1, int n1, const uint64_t* d2, int n2, int match_bits, float ratio, int32_t* pairs)
{
    int m = 0;
    if (n1 <= 0 || n2 <= 0) return 0;
    for (int i = 0; i < n1; ++i) {
        int bestIdx = -1, secondIdx = -1, bestDist = INT_MAX, secondDist = INT_MAX;
        for (int j = 0; j < n2; ++j) {
            int dist = hamming(d1 + 8 * (size_t)i, d2 + 8 * (size_t)j, match_bits);
            if (dist >= secondDist) continue;
            if (dist < bestDist) {
                secondDist = bestDist; secondIdx = bestIdx;
                bestDist = dist; bestIdx = j;
            } else if (dist < secondDist) {
                secondDist = dist; secondIdx = j;
            }
        }
        if (bestIdx != -1 && secondIdx != -1 && (float)bestDist < ratio * (float)secondDist) {
            pairs[2 * m] = i; pairs[2 * m + 1] = bestIdx; ++m;
        }
    }
    return m;
}

/* ========================================================================== */
/* RANSAC                                                                       */
/* ========================================================================== */

/* computeSampsonError, ransac.cpp:12-23.  p = (x1, y1, x2, y2). */
double voo_sampson(const double* F, const double* p)
{
    double x = p[0], y = p[1], xp = p[2], yp = p[3];
    double Fx0 = (F[0] * x + F[1] * y) + F[2] * 1.0;
    double Fx1 = (F[3] * x + F[4] * y) + F[5] * 1.0;
    double Ft0 = (F[0] * xp + F[3] * yp) + F[6] * 1.0;
    double Ft1 = (F[1] * xp + F[4] * yp) + F[7] * 1.0;
    double Ft2 = (F[2] * xp + F[5] * yp) + F[8] * 1.0;
    double v = (Ft0 * x + Ft1 * y) + Ft2 * 1.0;
    double num = v * v;
    double den = ((Fx0 * Fx0 + Fx1 * Fx1) + Ft0 * Ft0) + Ft1 * Ft1;
    if (den < 1e-12) return DBL_MAX;
    return num / den;
}

/* computeFundamentalMatrix on an 8-point minimal sample (ransac.cpp:63-93), sequential sums. */
int voo_fit_F8(const double* pts, const int32_t idx[8], double F[9])
{
    double mx1 = 0, my1 = 0, mx2 = 0, my2 = 0;
    for (int i = 0; i < 8; ++i) {
        const double* p = pts + 4 * (size_t)idx[i];
        mx1 = mx1 + p[0]; my1 = my1 + p[1]; mx2 = mx2 + p[2]; my2 = my2 + p[3];
    }
    mx1 = mx1 / 8.0; my1 = my1 / 8.0; mx2 = mx2 / 8.0; my2 = my2 / 8.0;
    double sc1 = 0, sc2 = 0;
    for (int i = 0; i < 8; ++i) {
        const double* p = pts + 4 * (size_t)idx[i];
        double a = p[0] - mx1, b = p[1] - my1, c = p[2] - mx2, d = p[3] - my2;
        sc1 = sc1 + (a * a + b * b);
        sc2 = sc2 + (c * c + d * d);
    }
    sc1 = sqrt(2.0) / sqrt(sc1 / 8.0);
    sc2 = sqrt(2.0) / sqrt(sc2 / 8.0);
    double o1x = -(sc1 * mx1), o1y = -(sc1 * my1), o2x = -(sc2 * mx2), o2y = -(sc2 * my2);
    double M[8][9];
    for (int i = 0; i < 8; ++i) {
        const double* p = pts + 4 * (size_t)idx[i];
        design_row(sc1 * p[0] + o1x, sc1 * p[1] + o1y, sc2 * p[2] + o2x, sc2 * p[3] + o2y, M[i]);
    }
    double f[9];
    nullvec_8x9(M, f);
    denormalize(f, sc1, mx1, my1, sc2, mx2, my2, F);
    rank2(F);
    return 0;
}

/* computeFundamentalMatrix on n >= 8 inliers (the refit, ransac.cpp:193): least-squares
 * null vector as the smallest eigenvector of A^T A; sums in the fixed device order. */
int voo_fit_F(const double* pts, const int32_t* idx, int n, double F[9])
{
    return voo_fit_F_warm(pts, idx, n, NULL, F);
}

int voo_fit_F_warm(const double* pts, const int32_t* idx, int n, const double* Fb, double F[9])
{
    if (n < 8) return -1;
    red256 r[4];
    double mean[4];
    for (int c = 0; c < 4; ++c) {
        for (int t = 0; t < VOO_RED_THREADS; ++t) {
            double s = 0.0;
            for (int i = t; i < n; i += VOO_RED_THREADS) s = s + pts[4 * (size_t)idx[i] + c];
            r[c].v[t] = s;
        }
        mean[c] = red_finish(&r[c]) / (double)n;
    }
    for (int g = 0; g < 2; ++g) {
        for (int t = 0; t < VOO_RED_THREADS; ++t) {
            double s = 0.0;
            for (int i = t; i < n; i += VOO_RED_THREADS) {
                const double* p = pts + 4 * (size_t)idx[i];
                double a = p[2 * g] - mean[2 * g], b = p[2 * g + 1] - mean[2 * g + 1];
                s = s + (a * a + b * b);
            }
            r[g].v[t] = s;
        }
    }
    double sc1 = sqrt(2.0) / sqrt(red_finish(&r[0]) / (double)n);
    double sc2 = sqrt(2.0) / sqrt(red_finish(&r[1]) / (double)n);
    double o1x = -(sc1 * mean[0]), o1y = -(sc1 * mean[1]), o2x = -(sc2 * mean[2]), o2y = -(sc2 * mean[3]);
    double AtA[81];
    static red256 acc[45];
    for (int t = 0; t < VOO_RED_THREADS; ++t) {
        double s[45];
        for (int e = 0; e < 45; ++e) s[e] = 0.0;
        for (int i = t; i < n; i += VOO_RED_THREADS) {
            const double* p = pts + 4 * (size_t)idx[i];
            double a[9];
            design_row(sc1 * p[0] + o1x, sc1 * p[1] + o1y, sc2 * p[2] + o2x, sc2 * p[3] + o2y, a);
            int e = 0;
            for (int u = 0; u < 9; ++u)
                for (int v = u; v < 9; ++v) { s[e] = s[e] + a[u] * a[v]; ++e; }
        }
        for (int e = 0; e < 45; ++e) acc[e].v[t] = s[e];
    }
    {
        int e = 0;
        for (int u = 0; u < 9; ++u)
            for (int v = u; v < 9; ++v) {
                double x = red_finish(&acc[e]); ++e;
                AtA[u * 9 + v] = x; AtA[v * 9 + u] = x;
            }
    }
    if (voo_dbg_capture_normal) memcpy(voo_dbg_capture_normal, AtA, sizeof(AtA));
    double f0[9], f[9];
    if (Fb) warm_start(Fb, sc1, mean[0], mean[1], sc2, mean[2], mean[3], f0);
    else for (int i = 0; i < 9; ++i) f0[i] = 1.0;
    ls_nullvec9(AtA, f0, f);
    memcpy(voo_dbg_refit_f, f, sizeof(f));
    denormalize(f, sc1, mean[0], mean[1], sc2, mean[2], mean[3], F);
    rank2(F);
    return 0;
}

/* test hook: the refit's normal matrix A^T A (voo_fit_F_warm's 45 sums, in its order) */
int voo_refit_normal(const double* pts, const int32_t* idx, int n, double AtA_out[81])
{
    if (n < 8) return -1;
    voo_dbg_capture_normal = AtA_out;
    double F[9];
    int rc = voo_fit_F_warm(pts, idx, n, NULL, F);
    voo_dbg_capture_normal = NULL;
    return rc;
}

/* Ransac::run, ransac.cpp:120-194, with the sampler of voo_sample8 and the chunk drop of
 * quirk 7: only matches [0, T*floor(m/T)) are scored. */
int voo_ransac(const double* pts, int m, double prob, double thr, int T, uint64_t seed,
               int32_t* counts, int32_t* inl_idx, voo_ransac_result* res)
{
    return voo_ransac_ex(pts, m, prob, thr, T, seed, 0, counts, inl_idx, res);
}

/* rng_mode 1: hypothesis k's sample is the k-th std::sample(data, 8, rng) of rng = std::mt19937(seed32),
 * seed32 = the low 32 bits of seed (ransac.cpp:137,142; vo_oracle_mt.cpp) */
int voo_ransac_ex(const double* pts, int m, double prob, double thr, int T, uint64_t seed, int rng_mode,
                  int32_t* counts, int32_t* inl_idx, voo_ransac_result* res)
{
    memset(res, 0, sizeof(*res));
    res->best_k = -1;
    if (m < 8 || T < 1) return -1;
    int32_t* tab = NULL;
    if (rng_mode == 1) {
        const int mi = voo_ransac_maxit_initial(prob), ntab = mi > 2000 ? mi : 2000;   /* clamp: <= 2000 later */
        tab = (int32_t*)malloc(sizeof(int32_t) * 8 * (size_t)ntab);
        voo_mt_samples((uint32_t)seed, m, ntab, tab);
    }
#define SAMPLE8(k, s8) do { if (tab) memcpy((s8), tab + 8 * (size_t)(k), 8 * sizeof(int32_t)); \
                            else voo_sample8(seed, (k), m, (s8)); } while (0)
    int chunk = m / T;
    int scored = chunk * T;
    int maxIt = voo_ransac_maxit_initial(prob);
    int best = 0, bestk = -1, it;
    double F[9];
    for (it = 0; it < maxIt; ++it) {
        int32_t s8[8];
        SAMPLE8(it, s8);
        voo_fit_F8(pts, s8, F);
        int c = 0;
        for (int i = 0; i < scored; ++i)
            if (voo_sampson(F, pts + 4 * (size_t)i) < thr) ++c;
        if (counts && it < 2000) counts[it] = c;
        if (c > best) {
            best = c; bestk = it;
            int u = voo_ransac_maxit_update(best, m, prob);
            if (u >= 0) maxIt = u;
        }
    }
    res->n_evaluated = it;
    res->best_k = bestk;
    res->best_count = best;
    if (bestk < 0) { res->n_inl = 0; res->fitted = 0; free(tab); return 0; }
    int32_t s8[8];
    SAMPLE8(bestk, s8);
    free(tab);
#undef SAMPLE8
    voo_fit_F8(pts, s8, F);
    int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * m);
    int n = 0;
    for (int i = 0; i < scored; ++i)
        if (voo_sampson(F, pts + 4 * (size_t)i) < thr) idx[n++] = i;
    res->n_inl = n;
    if (inl_idx) memcpy(inl_idx, idx, sizeof(int32_t) * n);
    if (n >= 8) { voo_fit_F_warm(pts, idx, n, F, res->F); res->fitted = 1; }
    free(idx);
    return 0;
}

/* ========================================================================== */
/* pose                                                                         */
/* ========================================================================== */

/* SVD of a 3x3 A (cv::SVD::compute of E, PoseUpdate.hpp:75-77): v3 = the smallest
 * eigenvector of A^T A (min_eigvec3), the other two from one 2x2 Jacobi rotation in the plane
 * orthogonal to v3; u_i = A v_i / s_i (i = 1, 2), u3 = u1 x u2.  Same code as k_refit. */
static void svd3(const double* A, double* U, double* S, double* Vt)
{
    double AtA[9], v3[3];
    mtm3(A, A, AtA);
    min_eigvec3(AtA, v3);
    /* orthonormal basis (p, q) of the plane orthogonal to v3: p = e_m x v3 / |.|, m the first
     * index of the smallest |v3_m|; q = v3 x p */
    int m = 0;
    if (fabs(v3[1]) < fabs(v3[m])) m = 1;
    if (fabs(v3[2]) < fabs(v3[m])) m = 2;
    double p[3];
    if (m == 0) { p[0] = 0.0; p[1] = -v3[2]; p[2] = v3[1]; }
    else if (m == 1) { p[0] = v3[2]; p[1] = 0.0; p[2] = -v3[0]; }
    else { p[0] = -v3[1]; p[1] = v3[0]; p[2] = 0.0; }
    const double rp = 1.0 / sqrt((p[0] * p[0] + p[1] * p[1]) + p[2] * p[2]);
    p[0] = p[0] * rp; p[1] = p[1] * rp; p[2] = p[2] * rp;
    double q[3] = {v3[1] * p[2] - v3[2] * p[1], v3[2] * p[0] - v3[0] * p[2], v3[0] * p[1] - v3[1] * p[0]};
    /* the 2x2 restriction of A^T A to that plane, diagonalized by one Jacobi rotation (the
     * rotation of the classic Jacobi eigenvalue method) */
    double Sp[3], Sq[3];
    for (int i = 0; i < 3; ++i) {
        Sp[i] = (AtA[i * 3 + 0] * p[0] + AtA[i * 3 + 1] * p[1]) + AtA[i * 3 + 2] * p[2];
        Sq[i] = (AtA[i * 3 + 0] * q[0] + AtA[i * 3 + 1] * q[1]) + AtA[i * 3 + 2] * q[2];
    }
    const double m00 = (p[0] * Sp[0] + p[1] * Sp[1]) + p[2] * Sp[2];
    const double m01 = (p[0] * Sq[0] + p[1] * Sq[1]) + p[2] * Sq[2];
    const double m11 = (q[0] * Sq[0] + q[1] * Sq[1]) + q[2] * Sq[2];
    double c = 1.0, s = 0.0, t = 0.0;
    if (m01 != 0.0) {
        const double theta = (m11 - m00) / (2.0 * m01);
        t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
        if (theta < 0.0) t = -t;
        c = 1.0 / sqrt(t * t + 1.0);
        s = t * c;
    }
    const double l1 = m00 - t * m01, l2 = m11 + t * m01;
    double w1[3], w2[3];
    for (int i = 0; i < 3; ++i) { w1[i] = c * p[i] - s * q[i]; w2[i] = s * p[i] + c * q[i]; }
    double V[9];                               /* columns: descending eigenvalue, then v3 */
    const double* va = l2 > l1 ? w2 : w1;
    const double* vb = l2 > l1 ? w1 : w2;
    for (int i = 0; i < 3; ++i) { V[i * 3 + 0] = va[i]; V[i * 3 + 1] = vb[i]; V[i * 3 + 2] = v3[i]; }
    double u[3][3];
    for (int cc = 0; cc < 2; ++cc) {
        double v0 = V[0 * 3 + cc], v1 = V[1 * 3 + cc], v2 = V[2 * 3 + cc];
        double a0 = (A[0] * v0 + A[1] * v1) + A[2] * v2;
        double a1 = (A[3] * v0 + A[4] * v1) + A[5] * v2;
        double a2 = (A[6] * v0 + A[7] * v1) + A[8] * v2;
        double sv = sqrt((a0 * a0 + a1 * a1) + a2 * a2);
        S[cc] = sv;
        if (sv > 0.0) { u[cc][0] = a0 / sv; u[cc][1] = a1 / sv; u[cc][2] = a2 / sv; }
        else { u[cc][0] = cc == 0 ? 1.0 : 0.0; u[cc][1] = cc == 1 ? 1.0 : 0.0; u[cc][2] = 0.0; }
    }
    {
        double a0 = (A[0] * v3[0] + A[1] * v3[1]) + A[2] * v3[2];
        double a1 = (A[3] * v3[0] + A[4] * v3[1]) + A[5] * v3[2];
        double a2 = (A[6] * v3[0] + A[7] * v3[1]) + A[8] * v3[2];
        S[2] = sqrt((a0 * a0 + a1 * a1) + a2 * a2);
    }
    u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
    u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
    u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
    for (int r = 0; r < 3; ++r)
        for (int cc = 0; cc < 3; ++cc) {
            U[r * 3 + cc] = u[cc][r];
            Vt[cc * 3 + r] = V[r * 3 + cc];
        }
}

/* smallest right singular vector of a 4x4 A (cv::triangulatePoints' SVD, last row of V^T):
 * the dominant eigenvector of adj(S), S = A^T A (the adjugate of a PSD S has S's
 * eigenvectors, eigenvalue of the smallest one the largest).  adj(S) is squared four times
 * (each power first scaled by the power of two bringing its largest diagonal entry into
 * [0.5, 1)), started from its column with the largest diagonal entry, power-iterated until
 * the unit iterate moves by <= 4e-16 (at most 16 steps).  k_triangulate runs the same code
 * per thread.  S of rank <= 2 (adj(S) = 0: no unique point) gives (0,0,0,1), a point that
 * fails the depth test. */
static void cof4_sym(const double* S, double* B)   /* B = adj(S), S symmetric: cofactors C_ij, i <= j */
{
    for (int i = 0; i < 4; ++i)
        for (int j = i; j < 4; ++j) {
            double m[9];
            int e = 0;
            for (int r = 0; r < 4; ++r) {
                if (r == j) continue;              /* adj = C^T: row j, column i of S removed */
                for (int c = 0; c < 4; ++c)
                    if (c != i) m[e++] = S[r * 4 + c];
            }
            double v = det3(m);
            if ((i + j) & 1) v = -v;
            B[i * 4 + j] = v; B[j * 4 + i] = v;
        }
}
static double pow2_scale4(const double* B)
{
    double m = 0.0;
    for (int i = 0; i < 4; ++i) if (B[i * 4 + i] > m) m = B[i * 4 + i];
    int e;
    (void)frexp(m, &e);
    return ldexp(1.0, -e);
}
static void nullvec4(const double* A, double* x)
{
    double S[16], B[16], B2[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            S[i * 4 + j] = ((A[0 * 4 + i] * A[0 * 4 + j] + A[1 * 4 + i] * A[1 * 4 + j]) + A[2 * 4 + i] * A[2 * 4 + j]) +
                           A[3 * 4 + i] * A[3 * 4 + j];
    cof4_sym(S, B);
    int k = 0;
    for (int i = 1; i < 4; ++i) if (B[i * 4 + i] > B[k * 4 + k]) k = i;
    if (!(B[k * 4 + k] > 0.0)) { x[0] = 0.0; x[1] = 0.0; x[2] = 0.0; x[3] = 1.0; return; }
    for (int q = 0; q < 4; ++q) {
        double r = pow2_scale4(B);
        for (int i = 0; i < 4; ++i)
            for (int j = i; j < 4; ++j) {
                double v = 0.0;
                for (int t = 0; t < 4; ++t) v = v + (B[i * 4 + t] * r) * (B[t * 4 + j] * r);
                B2[i * 4 + j] = v; B2[j * 4 + i] = v;
            }
        memcpy(B, B2, sizeof(B2));
    }
    k = 0;
    for (int i = 1; i < 4; ++i) if (B[i * 4 + i] > B[k * 4 + k]) k = i;
    double y[4], nn = 0.0;
    for (int i = 0; i < 4; ++i) { y[i] = B[i * 4 + k]; nn = nn + y[i] * y[i]; }
    double rn = 1.0 / sqrt(nn);
    for (int i = 0; i < 4; ++i) x[i] = y[i] * rn;
    for (int it = 0; it < 16; ++it) {
        double z[4], dot = 0.0;
        nn = 0.0;
        for (int i = 0; i < 4; ++i) {
            z[i] = ((B[i * 4 + 0] * x[0] + B[i * 4 + 1] * x[1]) + B[i * 4 + 2] * x[2]) + B[i * 4 + 3] * x[3];
            nn = nn + z[i] * z[i];
            dot = dot + z[i] * x[i];
        }
        double rs = (dot < 0.0 ? -1.0 : 1.0) / sqrt(nn);
        double diff = 0.0;
        for (int i = 0; i < 4; ++i) {
            double xn = z[i] * rs;
            double dd = fabs(xn - x[i]);
            if (dd > diff) diff = dd;
            x[i] = xn;
        }
        if (diff <= 4e-16) break;
    }
}

/* PoseUpdate::getPose (PoseUpdate.hpp:61-179). p1/p2: n x 2 f32 (cv::Point2f inliers). */
int voo_pose(const double* F, const double* K, const float* p1, const float* p2, int n, double scale,
             double* Rout, double* tout, int* counts4)
{
    double E[9], G[9];
    mtm3(K, F, G);                 /* K^T F */
    mm3(G, K, E);                  /* (K^T F) K */
    double nn = 0.0;
    for (int i = 0; i < 9; ++i) nn = nn + E[i] * E[i];
    nn = sqrt(nn);
    double inv = 1.0 / nn;
    int nz = 0;
    for (int i = 0; i < 9; ++i) { E[i] = E[i] * inv; nz += (E[i] != 0.0); }
    if (nz < 5) return VOO_ERR_DEGENERATE_E;       /* PoseUpdate.hpp:71-73 */
    double U[9], S[3], Vt[9];
    svd3(E, U, S, Vt);
    if (det3(U) < 0) for (int i = 0; i < 9; ++i) U[i] = -U[i];
    if (det3(Vt) < 0) for (int i = 0; i < 9; ++i) Vt[i] = -Vt[i];
    static const double W[9] = {0, -1, 0, 1, 0, 0, 0, 0, 1};
    static const double Wt[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1};
    double R1[9], R2[9], T[9];
    mm3(U, W, T); mm3(T, Vt, R1);
    mm3(U, Wt, T); mm3(T, Vt, R2);
    if (det3(R1) < 0) for (int i = 0; i < 9; ++i) R1[i] = -R1[i];
    if (det3(R2) < 0) for (int i = 0; i < 9; ++i) R2[i] = -R2[i];
    double t[3] = {U[2], U[5], U[8]};
    const double* Rc[4] = {R1, R1, R2, R2};
    const double sg[4] = {1.0, -1.0, 1.0, -1.0};
    double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    double ifx = 1.0 / fx, ify = 1.0 / fy;
    int maxPos = -1, bestc = 0;
    for (int cnd = 0; cnd < 4; ++cnd) {
        const double* R = Rc[cnd];
        double tc[3] = {t[0] * sg[cnd], t[1] * sg[cnd], t[2] * sg[cnd]};
        int cnt = 0;
        for (int i = 0; i < n; ++i) {
            /* cv::undistortPoints(K, no distortion): x = (u - cx) * (1/fx), stored f32 */
            float x1 = (float)(((double)p1[2 * i] - cx) * ifx), y1 = (float)(((double)p1[2 * i + 1] - cy) * ify);
            float x2 = (float)(((double)p2[2 * i] - cx) * ifx), y2 = (float)(((double)p2[2 * i + 1] - cy) * ify);
            double X1 = x1, Y1 = y1, X2 = x2, Y2 = y2;
            /* cvTriangulatePoints rows: x*P[2,k] - P[0,k], y*P[2,k] - P[1,k]; P1 = [I|0], P2 = [R|t] */
            double A[16];
            double P1[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
            double P2[12] = {R[0], R[1], R[2], tc[0], R[3], R[4], R[5], tc[1], R[6], R[7], R[8], tc[2]};
            for (int k = 0; k < 4; ++k) {
                A[0 * 4 + k] = X1 * P1[8 + k] - P1[0 + k];
                A[1 * 4 + k] = Y1 * P1[8 + k] - P1[4 + k];
                A[2 * 4 + k] = X2 * P2[8 + k] - P2[0 + k];
                A[3 * 4 + k] = Y2 * P2[8 + k] - P2[4 + k];
            }
            double X[4];
            nullvec4(A, X);
            /* points4D is CV_32F (type of the input points) */
            double h[4] = {(double)(float)X[0], (double)(float)X[1], (double)(float)X[2], (double)(float)X[3]};
            double w = h[3];
            if (fabs(w) < 1e-6) continue;
            double iw = 1.0 / w;
            double Xh0 = h[0] * iw, Xh1 = h[1] * iw, Xh2 = h[2] * iw;
            double z1 = Xh2;
            double z2 = ((R[6] * Xh0 + R[7] * Xh1) + R[8] * Xh2) + tc[2];
            if (z1 > 0 && z2 > 0) ++cnt;
        }
        if (counts4) counts4[cnd] = cnt;
        if (cnt > maxPos) { maxPos = cnt; bestc = cnd; }
    }
    const double* Rf = Rc[bestc];
    double tf[3] = {t[0] * sg[bestc], t[1] * sg[bestc], t[2] * sg[bestc]};
    double Rfin[9];
    memcpy(Rfin, Rf, sizeof(Rfin));
    if (det3(Rfin) < 0) for (int i = 0; i < 9; ++i) Rfin[i] = -Rfin[i];
    double tn = sqrt((tf[0] * tf[0] + tf[1] * tf[1]) + tf[2] * tf[2]);
    if (tn > 1e-6) {
        double f = scale / tn;
        tf[0] = tf[0] * f; tf[1] = tf[1] * f; tf[2] = tf[2] * f;
    }
    memcpy(Rout, Rfin, sizeof(Rfin));
    memcpy(tout, tf, sizeof(tf));
    return VOO_OK;
}

/* ========================================================================== */
/* trajectory loop                                                              */
/* ========================================================================== */

struct voo_vo {
    voo_config c;
    int64_t frame;
    int have_prev;
    int n_prev;
    int32_t* kps_prev; uint64_t* desc_prev;
    int32_t* kps_cur; uint64_t* desc_cur;
    int model_n; double model_F[9]; float* model_p1; float* model_p2;
    double Tcurr[16];
    int last_valid;
};

voo_vo* voo_vo_create(const voo_config* c)
{
    voo_vo* s = (voo_vo*)calloc(1, sizeof(voo_vo));
    s->c = *c;
    int N = c->max_kpts;
    s->kps_prev = (int32_t*)malloc(sizeof(int32_t) * 2 * N);
    s->kps_cur = (int32_t*)malloc(sizeof(int32_t) * 2 * N);
    s->desc_prev = (uint64_t*)malloc(sizeof(uint64_t) * 8 * N);
    s->desc_cur = (uint64_t*)malloc(sizeof(uint64_t) * 8 * N);
    s->model_p1 = (float*)malloc(sizeof(float) * 2 * N);
    s->model_p2 = (float*)malloc(sizeof(float) * 2 * N);
    for (int i = 0; i < 16; ++i) s->Tcurr[i] = (i % 5 == 0) ? 1.0 : 0.0;
    return s;
}

void voo_vo_destroy(voo_vo* s)
{
    if (!s) return;
    free(s->kps_prev); free(s->kps_cur); free(s->desc_prev); free(s->desc_cur);
    free(s->model_p1); free(s->model_p2); free(s);
}

static void mm4(const double* A, const double* B, double* C)
{
    double T[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            T[i * 4 + j] = ((A[i * 4 + 0] * B[0 * 4 + j] + A[i * 4 + 1] * B[1 * 4 + j]) + A[i * 4 + 2] * B[2 * 4 + j]) +
                           A[i * 4 + 3] * B[3 * 4 + j];
    memcpy(C, T, sizeof(T));
}

/* 4x4 inverse by Gauss-Jordan with partial pivoting (cv::Mat::inv, DECOMP_LU). */
static void inv4(const double* M, double* Inv)
{
    double a[4][8];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) a[i][j] = j < 4 ? M[i * 4 + j] : (j - 4 == i ? 1.0 : 0.0);
    for (int c = 0; c < 4; ++c) {
        int p = c;
        for (int r = c + 1; r < 4; ++r) if (fabs(a[r][c]) > fabs(a[p][c])) p = r;
        if (p != c) for (int j = 0; j < 8; ++j) { double t = a[c][j]; a[c][j] = a[p][j]; a[p][j] = t; }
        double pv = a[c][c];
        for (int j = 0; j < 8; ++j) a[c][j] = a[c][j] / pv;
        for (int r = 0; r < 4; ++r) {
            if (r == c) continue;
            double f = a[r][c];
            for (int j = 0; j < 8; ++j) a[r][j] = a[r][j] - f * a[c][j];
        }
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) Inv[i * 4 + j] = a[i][j + 4];
}

/* ||t(gt[i]^-1 gt[last])||  (VisualOdometry.cpp:161-162) */
static double gt_scale(const double* gt, int gt_n, int64_t i, int last)
{
    if (!gt || i >= gt_n || last >= gt_n) return 1.0;
    double Gi[16], Gl[16], Ii[16], Tr[16];
    for (int r = 0; r < 16; ++r) { Gi[r] = r < 12 ? gt[12 * i + r] : (r == 15 ? 1.0 : 0.0); Gl[r] = r < 12 ? gt[12 * (size_t)last + r] : (r == 15 ? 1.0 : 0.0); }
    inv4(Gi, Ii);
    mm4(Ii, Gl, Tr);
    return sqrt((Tr[3] * Tr[3] + Tr[7] * Tr[7]) + Tr[11] * Tr[11]);
}

static void push_pose(const double* T, int flip, double* out)
{
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) out[r * 4 + c] = (flip && r == 2) ? -T[r * 4 + c] : T[r * 4 + c];
}

int voo_vo_process(voo_vo* s, const uint8_t* gray, size_t stride, const double* gt, int gt_n,
                   double pose_out[12], int* status, int32_t* info)
{
    const voo_config* c = &s->c;
    int64_t fi = s->frame++;
    if (info) { memset(info, 0, 8 * sizeof(int32_t)); info[3] = -1; }
    if (fi == 0) {
        /* VisualOdometry.cpp:56-66: frame 0 pushed as identity (no flipZ) */
        push_pose(s->Tcurr, 0, pose_out);
        *status = VO_STATUS_FIRST;
        if (gray) {
            s->n_prev = voo_extract(c, gray, stride, s->kps_prev, s->desc_prev, NULL);
            s->have_prev = 1;
        }
        if (info) info[0] = s->n_prev;
        return 0;
    }
    if (!gray) { push_pose(s->Tcurr, 0, pose_out); *status = VO_STATUS_MISSING; return 0; }  /* :77-82 */
    int n = voo_extract(c, gray, stride, s->kps_cur, s->desc_cur, NULL);
    int32_t* pairs = (int32_t*)malloc(sizeof(int32_t) * 2 * (s->n_prev > 0 ? s->n_prev : 1));
    int m;
    STAGE(VOO_STAGE_MATCH, m = voo_match(s->desc_prev, s->n_prev, s->desc_cur, n, c->match_bits, c->ratio, pairs));
    if (info) { info[0] = n; info[1] = m; }
    if (m < 8) {                                                  /* :108-115 */
        free(pairs);
        push_pose(s->Tcurr, 1, pose_out); *status = VO_STATUS_FEW_MATCHES; return 0;
    }
    double* pts = (double*)malloc(sizeof(double) * 4 * m);
    for (int k = 0; k < m; ++k) {                                 /* :117-123 */
        const int32_t* a = s->kps_prev + 2 * pairs[2 * k];
        const int32_t* b = s->kps_cur + 2 * pairs[2 * k + 1];
        pts[4 * k] = a[0]; pts[4 * k + 1] = a[1]; pts[4 * k + 2] = b[0]; pts[4 * k + 3] = b[1];
    }
    free(pairs);
    voo_ransac_result rr;
    int32_t* inl = (int32_t*)malloc(sizeof(int32_t) * m);
    STAGE(VOO_STAGE_RANSAC, voo_ransac_ex(pts, m, c->ransac_p, c->sampson_thr, c->ransac_chunk_threads,
                                           voo_frame_seed(c->seed, fi), c->rng_mode, NULL, inl, &rr));
    if (info) { info[2] = rr.n_inl; info[3] = rr.best_k; info[4] = rr.n_evaluated; info[5] = rr.fitted; }
    if (rr.fitted) {                                              /* model state leak, quirk 9 */
        memcpy(s->model_F, rr.F, sizeof(rr.F));
        s->model_n = rr.n_inl;
        for (int k = 0; k < rr.n_inl; ++k) {
            const double* p = pts + 4 * (size_t)inl[k];
            s->model_p1[2 * k] = (float)p[0]; s->model_p1[2 * k + 1] = (float)p[1];
            s->model_p2[2 * k] = (float)p[2]; s->model_p2[2 * k + 1] = (float)p[3];
        }
    }
    free(inl); free(pts);
    if (s->model_n < 8) {                                         /* :147-153 */
        push_pose(s->Tcurr, 1, pose_out); *status = VO_STATUS_FEW_INLIERS; return 0;
    }
    double scale = gt_scale(gt, gt_n, fi, s->last_valid);
    s->last_valid = (int)fi;                                      /* :163-166 */
    { int32_t* t = s->kps_prev; s->kps_prev = s->kps_cur; s->kps_cur = t; }
    { uint64_t* t = s->desc_prev; s->desc_prev = s->desc_cur; s->desc_cur = t; }
    s->n_prev = n;
    double R[9], t[3];
    int rc;
    STAGE(VOO_STAGE_POSE, rc = voo_pose(s->model_F, c->K, s->model_p1, s->model_p2, s->model_n, scale, R, t, NULL));
    if (rc != VOO_OK) { push_pose(s->Tcurr, 1, pose_out); *status = VO_STATUS_DEGENERATE; return rc; }
    double Trel[16] = {R[0], R[1], R[2], t[0], R[3], R[4], R[5], t[1], R[6], R[7], R[8], t[2], 0, 0, 0, 1};
    mm4(s->Tcurr, Trel, s->Tcurr);                                /* :180 */
    push_pose(s->Tcurr, 1, pose_out);
    *status = VO_STATUS_OK;
    return 0;
}

void voo_config_default(voo_config* c, int width, int height)
{
    memset(c, 0, sizeof(*c));
    c->width = width; c->height = height;
    c->max_kpts = 2000; c->nms_k = 3; c->resp_thr = 20000.0f;
    c->border_row = 35; c->border_col = 37;
    c->ratio = 0.75f; c->match_bits = 32;
    c->ransac_p = 0.99; c->sampson_thr = 1.0; c->ransac_chunk_threads = 8;
    c->seed = 0xACE0ULL;
    double K[9] = {7.188560000000e+02, 0, 6.071928000000e+02, 0, 7.188560000000e+02, 1.852157000000e+02, 0, 0, 1.0};
    memcpy(c->K, K, sizeof(K));
}

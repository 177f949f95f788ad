// vo_kernels.hip -- gfx950 (CDNA4) kernels of the extract -> match -> pose hot path.
//
// Arithmetic contract: compiled with -ffp-contract=off; f32/f64 '/' and sqrt are the
// correctly rounded HIP defaults; every expression is written in the operation order
// of oracle/vo_oracle.c (which cites the reference file:line it restates), so keypoints,
// descriptor bits, matches, per-hypothesis inlier counts, F, R and t are bit-identical
// to the CPU oracle on the same inputs.  No MFMA: the path is stencil / bit-count /
// small-f64 bound, and a matrix-core matcher co-running with k_stencil perturbed the stencil's
// packed-FP32 results in lanes 32-63 ("Matrix cores and the stencil"), so
// none ships (tests/test_no_mfma.py checks the code object).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include <utility>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "vo_internal.h"
#include "vo_sampson32.h"
#include "../../include/vo_freak_tables.h"
#include "../../include/vo_mi355x.h"

namespace vo {

// ---------------------------------------------------------------------------
// constant tables
// ---------------------------------------------------------------------------
// per pair t and component c = x, y: the unit direction d_c/|d| split into A_c = f32(d_c/|d|) and
// B_c = f32(d_c/|d| - A_c) (|d| the reference's f32 norm, the quotient in f64).
// (ic*d_c)/|d| in f32 == fmaf(ic, A_c, ic * B_c) for every ic in [-255,255], every pair and both
// components (tests/test_describe_division.py, exhaustive; up to the sign of a zero term): one
// product and one fma per term and component instead of two products and an fma
// Rows p of the pair order padded to whole groups of DS_OG terms with zero terms (dx = dy = 0:
// the term is a zero, which leaves a sum that is never -0 unchanged), so the describe loop has
// no remainder iterations.
#ifndef DS_OG
#define DS_OG 8
#endif
#define DS_OROWS (VO_FREAK_NPOINTS + DS_OG - 1)     // sample rows incl. the zero padding rows
constexpr int ds_onpad()                            // sum over p of ceil((42 - p) / OG) * OG (1056 at 8)
{
    int n = 0;
    for (int k = 1; k < VO_FREAK_NPOINTS; ++k) n += (k + DS_OG - 1) / DS_OG * DS_OG;
    return n;
}
#define DS_ONPAD (ds_onpad())
__constant__ float4 c_orient[DS_ONPAD];
// the same entries unpadded, in pair order (the fully unrolled describe, DS_UNROLL), plus one
// block of zeros read by the last block's prefetch
#ifndef DS_UB
#define DS_UB 8                // terms per block of the unrolled sum (one table request per block)
#endif
__constant__ float4 c_orient_u[VO_FREAK_NPAIRS + DS_UB];
// the pattern points (x, y) and the pair list (p, q) in pair order (k_describe_pf's loop indices)
__constant__ short2 c_ppt[VO_FREAK_NPOINTS];
__constant__ uchar2 c_pair[VO_FREAK_NPAIRS];
// k_describe_pf's term tables, padded to whole 64-term chunks (padding: both rows 0, weights 0):
// each entry one scalar load -- the pair as the two sample rows' LDS byte offsets (p * 256 |
// q * 256 << 16), the weights as in c_orient_u
#ifndef DP_CHUNK
#define DP_CHUNK 96                    // k_describe_pf: terms per chunk of its LDS ring (64: 1.3-2.6 us slower per call, r5q)
#endif
#define DP_NPAD (((VO_FREAK_NPAIRS + DP_CHUNK - 1) / DP_CHUNK) * DP_CHUNK)
__constant__ uint32_t c_pairoff[DP_NPAD];
__constant__ float4 c_orient_pf[DP_NPAD];

static bool g_tables_ready = false;
static void ensure_tables()
{
    if (g_tables_ready) return;
    int8_t px[VO_FREAK_NPOINTS], py[VO_FREAK_NPOINTS];
    uint8_t pp[VO_FREAK_NPAIRS], pq[VO_FREAK_NPAIRS];
    for (int i = 0; i < VO_FREAK_NPOINTS; ++i) { px[i] = (int8_t)vo_freak_points[i][0]; py[i] = (int8_t)vo_freak_points[i][1]; }
    int e = 0;
    for (int p = 0; p < VO_FREAK_NPOINTS; ++p)
        for (int q = p + 1; q < VO_FREAK_NPOINTS; ++q) { pp[e] = (uint8_t)p; pq[e] = (uint8_t)q; ++e; }
    static float4 orient[DS_ONPAD];
    static float4 orient_u[VO_FREAK_NPAIRS + DS_UB];
    int o = 0;
    for (int t = 0; t < VO_FREAK_NPAIRS; ++t) {
        const float dx = (float)(px[pp[t]] - px[pq[t]]), dy = (float)(py[pp[t]] - py[pq[t]]);
        const float nrm = sqrtf(dx * dx + dy * dy);    // host sqrtf: correctly rounded
        const double ux = (double)dx / (double)nrm, uy = (double)dy / (double)nrm;
        const float ax = (float)ux, ay = (float)uy;
        orient_u[t] = make_float4(ax, ay, (float)(ux - (double)ax), (float)(uy - (double)ay));
        orient[o++] = orient_u[t];
        if (pq[t] == VO_FREAK_NPOINTS - 1)             // end of row p: pad to a whole group
            while (o % DS_OG) orient[o++] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    if (o != DS_ONPAD) fprintf(stderr, "[vo_mi355x] orientation table size %d != %d\n", o, DS_ONPAD);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_orient), orient, sizeof(orient));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_orient_u), orient_u, sizeof(orient_u));
    static short2 ppt[VO_FREAK_NPOINTS];
    static uchar2 pair[VO_FREAK_NPAIRS];
    for (int i = 0; i < VO_FREAK_NPOINTS; ++i) ppt[i] = make_short2(px[i], py[i]);
    for (int t = 0; t < VO_FREAK_NPAIRS; ++t) pair[t] = make_uchar2(pp[t], pq[t]);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_ppt), ppt, sizeof(ppt));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_pair), pair, sizeof(pair));
    static uint32_t pairoff[DP_NPAD];
    static float4 orient_pf[DP_NPAD];
    for (int t = 0; t < DP_NPAD; ++t) {
        pairoff[t] = t < VO_FREAK_NPAIRS ? (uint32_t)pp[t] * 256u | ((uint32_t)pq[t] * 256u) << 16 : 0u;
        orient_pf[t] = t < VO_FREAK_NPAIRS ? orient_u[t] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_pairoff), pairoff, sizeof(pairoff));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_orient_pf), orient_pf, sizeof(orient_pf));
    g_tables_ready = true;
}

// ---------------------------------------------------------------------------
// deterministic math (mirror of oracle/vo_oracle.c, same constants, same order)
// ---------------------------------------------------------------------------
__device__ __constant__ double c_atan_hi[9] = {
    0.0, 0.12435499454676144, 0.24497866312686414, 0.35877067027057225,
    0.4636476090008061, 0.5585993153435624, 0.6435011087932844,
    0.7188299996216245, 0.7853981633974483};
__device__ __constant__ double c_atan_lo[9] = {
    0.0, -3.1253241424539383e-18, 1.0698755618734451e-17, -2.4623815582638635e-17,
    2.2698777452961687e-17, -5.4556305485916264e-18, 1.5834785051444286e-17,
    -2.1478388444456983e-17, 3.061616997868383e-17};

__device__ __forceinline__ bool sgnbit(double x) { return (__double_as_longlong(x) >> 63) != 0; }

__device__ double det_atan01(double r)
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
    return c_atan_hi[i] + (az + c_atan_lo[i]);
}

__device__ double det_atan2(double y, double x)
{
    const double PI_HI = 3.141592653589793, PI_LO = 1.2246467991473532e-16;
    const double PIO2_HI = 1.5707963267948966, PIO2_LO = 6.123233995736766e-17;
    double ax = fabs(x), ay = fabs(y), t;
    if (ay == 0.0 && ax == 0.0) {
        t = sgnbit(x) ? PI_HI : 0.0;
    } else if (ay > ax) {
        double b = det_atan01(ax / ay);
        t = sgnbit(x) ? (PIO2_HI + b) + PIO2_LO : (PIO2_HI - b) + PIO2_LO;
    } else {
        double b = det_atan01(ay / ax);
        t = sgnbit(x) ? (PI_HI - b) + PI_LO : b;
    }
    if (sgnbit(y)) t = -t;
    return t;
}

__device__ void det_sincos(double x, double* s_out, double* c_out)
{
    const double PIO2_1 = 1.570796325802803, PIO2_2 = 9.920935791635221e-10,
                 PIO2_3 = 5.170182981794105e-19, TWO_OVER_PI = 0.6366197723675814;
    double kf = floor(x * TWO_OVER_PI + 0.5);
    int k = (int)kf;
    double r = ((x - kf * PIO2_1) - kf * PIO2_2) - kf * PIO2_3;
    double r2 = r * r;
    double ps = -1.0 / 355687428096000.0;
    ps = ps * r2 + 1.0 / 1307674368000.0;
    ps = ps * r2 - 1.0 / 6227020800.0;
    ps = ps * r2 + 1.0 / 39916800.0;
    ps = ps * r2 - 1.0 / 362880.0;
    ps = ps * r2 + 1.0 / 5040.0;
    ps = ps * r2 - 1.0 / 120.0;
    ps = ps * r2 + 1.0 / 6.0;
    double sr = r - r * (r2 * ps);
    double pc = 1.0 / 6402373705728000.0;
    pc = pc * r2 - 1.0 / 20922789888000.0;
    pc = pc * r2 + 1.0 / 87178291200.0;
    pc = pc * r2 - 1.0 / 479001600.0;
    pc = pc * r2 + 1.0 / 3628800.0;
    pc = pc * r2 - 1.0 / 40320.0;
    pc = pc * r2 + 1.0 / 720.0;
    pc = pc * r2 - 1.0 / 24.0;
    pc = pc * r2 + 0.5;
    double cr = 1.0 - r2 * pc;
    switch (k & 3) {
    case 0: *s_out = sr;  *c_out = cr;  break;
    case 1: *s_out = cr;  *c_out = -sr; break;
    case 2: *s_out = -sr; *c_out = -cr; break;
    default: *s_out = -cr; *c_out = sr; break;
    }
}

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// voo_sample8: Floyd's algorithm + insertion sort (oracle/vo_oracle.c).
__device__ void sample8(uint64_t seed, int k, int m, int out[8])
{
    uint64_t st = mix64(seed ^ (0x9E3779B97F4A7C15ULL * (uint64_t)(k + 1)));
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        int j = m - 8 + c;
        st += 0x9E3779B97F4A7C15ULL;
        uint64_t r = mix64(st);
        int t = (int)__umul64hi(r, (uint64_t)(j + 1));
        bool present = false;
#pragma unroll
        for (int i = 0; i < c; ++i) present |= (out[i] == t);
        out[c] = present ? j : t;
    }
    // insertion sort with static indices (sorting network of adjacent swaps, same result)
#pragma unroll
    for (int i = 1; i < 8; ++i) {
#pragma unroll
        for (int j = i; j > 0; --j) {
            int a = out[j - 1], b = out[j];
            bool sw = a > b;
            out[j - 1] = sw ? b : a;
            out[j] = sw ? a : b;
        }
    }
}

// ---------------------------------------------------------------------------
// small dense linear algebra (mirror of oracle/vo_oracle.c)
// ---------------------------------------------------------------------------

template <int n>
__device__ __forceinline__ int argmin_diag(const double* A)
{
    int b = 0;
#pragma unroll
    for (int i = 1; i < n; ++i)
        if (A[i * n + i] < A[b * n + b]) b = i;
    return b;
}

__device__ __forceinline__ void mm3(const double* A, const double* B, double* C)
{
    double T[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            T[i * 3 + j] = (A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j]) + A[i * 3 + 2] * B[2 * 3 + j];
#pragma unroll
    for (int i = 0; i < 9; ++i) C[i] = T[i];
}
__device__ __forceinline__ void mtm3(const double* A, const double* B, double* C)
{
    double T[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            T[i * 3 + j] = (A[0 * 3 + i] * B[0 * 3 + j] + A[1 * 3 + i] * B[1 * 3 + j]) + A[2 * 3 + i] * B[2 * 3 + j];
#pragma unroll
    for (int i = 0; i < 9; ++i) C[i] = T[i];
}
__device__ __forceinline__ double det3(const double* M)
{
    return (M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6])) +
           M[2] * (M[3] * M[7] - M[4] * M[6]);
}

// smallest eigenvector of a 3x3 symmetric PSD S via adj(S) (mirror of oracle min_eigvec3)
__device__ void min_eigvec3(const double* S, double* v)
{
    double B[9];
    B[0] = S[4] * S[8] - S[5] * S[7];
    B[4] = S[0] * S[8] - S[2] * S[6];
    B[8] = S[0] * S[4] - S[1] * S[3];
    B[1] = -(S[3] * S[8] - S[5] * S[6]); B[3] = B[1];
    B[2] = S[3] * S[7] - S[4] * S[6];    B[6] = B[2];
    B[5] = -(S[0] * S[7] - S[1] * S[6]); B[7] = B[5];
    double bmax = B[0];
    bmax = B[4] > bmax ? B[4] : bmax;
    bmax = B[8] > bmax ? B[8] : bmax;
    if (!(bmax > 0.0)) { v[0] = 0.0; v[1] = 0.0; v[2] = 1.0; return; }
#pragma unroll 1
    for (int q = 0; q < 4; ++q) {
        double m = 0.0;
#pragma unroll
        for (int i = 0; i < 3; ++i) m = B[i * 3 + i] > m ? B[i * 3 + i] : m;
        int e;
        (void)frexp(m, &e);
        const double r = ldexp(1.0, -e);
        double B2[9];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = i; j < 3; ++j) {
                const double x = ((B[i * 3 + 0] * r) * (B[0 * 3 + j] * r) + (B[i * 3 + 1] * r) * (B[1 * 3 + j] * r)) +
                                 (B[i * 3 + 2] * r) * (B[2 * 3 + j] * r);
                B2[i * 3 + j] = x; B2[j * 3 + i] = x;
            }
#pragma unroll
        for (int i = 0; i < 9; ++i) B[i] = B2[i];
    }
    int k = 0;
#pragma unroll
    for (int i = 1; i < 3; ++i) if (B[i * 3 + i] > B[k * 3 + k]) k = i;
    double c0 = B[0], c1 = B[3], c2 = B[6];
    if (k == 1) { c0 = B[1]; c1 = B[4]; c2 = B[7]; }
    if (k == 2) { c0 = B[2]; c1 = B[5]; c2 = B[8]; }
    const double nn = (c0 * c0 + c1 * c1) + c2 * c2;
    const double rn = 1.0 / sqrt(nn);
    v[0] = c0 * rn; v[1] = c1 * rn; v[2] = c2 * rn;
    for (int it = 0; it < 32; ++it) {
        double z[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) z[i] = (B[i * 3 + 0] * v[0] + B[i * 3 + 1] * v[1]) + B[i * 3 + 2] * v[2];
        const double zz = (z[0] * z[0] + z[1] * z[1]) + z[2] * z[2];
        const double dot = (z[0] * v[0] + z[1] * v[1]) + z[2] * v[2];
        const double rs = (dot < 0.0 ? -1.0 : 1.0) / sqrt(zz);
        double diff = 0.0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double xn = z[i] * rs;
            const double dd = fabs(xn - v[i]);
            if (dd > diff) diff = dd;
            v[i] = xn;
        }
        if (diff <= 4e-16) break;
    }
}

__device__ void rank2(double* F)
{
    double FtF[9], v[3];
    mtm3(F, F, FtF);
    min_eigvec3(FtF, v);
    const double v0 = v[0], v1 = v[1], v2 = v[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double fv = (F[i * 3 + 0] * v0 + F[i * 3 + 1] * v1) + F[i * 3 + 2] * v2;
        F[i * 3 + 0] = F[i * 3 + 0] - fv * v0;
        F[i * 3 + 1] = F[i * 3 + 1] - fv * v1;
        F[i * 3 + 2] = F[i * 3 + 2] - fv * v2;
    }
}

__device__ __forceinline__ void denormalize(const double* F0, double s1, double mx1, double my1,
                                            double s2, double mx2, double my2, double* F)
{
    double T1[9] = {s1, 0.0, -(s1 * mx1), 0.0, s1, -(s1 * my1), 0.0, 0.0, 1.0};
    double T2[9] = {s2, 0.0, -(s2 * mx2), 0.0, s2, -(s2 * my2), 0.0, 0.0, 1.0};
    double G[9];
    mtm3(T2, F0, G);
    mm3(G, T1, F);
}

__device__ __forceinline__ void design_row(double p1x, double p1y, double p2x, double p2y, double* a)
{
    a[0] = p1x * p2x; a[1] = p1x * p2y; a[2] = p1x;
    a[3] = p1y * p2x; a[4] = p1y * p2y; a[5] = p1y;
    a[6] = p2x; a[7] = p2y; a[8] = 1.0;
}

// computeSampsonError, ransac.cpp:12-23 (mirror of voo_sampson)
__device__ __forceinline__ double sampson(const double* F, double x, double y, double xp, double yp)
{
    double Fx0 = (F[0] * x + F[1] * y) + F[2] * 1.0;
    double Fx1 = (F[3] * x + F[4] * y) + F[5] * 1.0;
    double Ft0 = (F[0] * xp + F[3] * yp) + F[6] * 1.0;
    double Ft1 = (F[1] * xp + F[4] * yp) + F[7] * 1.0;
    double Ft2 = (F[2] * xp + F[5] * yp) + F[8] * 1.0;
    double v = (Ft0 * x + Ft1 * y) + Ft2 * 1.0;
    double num = v * v;
    double den = ((Fx0 * Fx0 + Fx1 * Fx1) + Ft0 * Ft0) + Ft1 * Ft1;
    if (den < 1e-12) return 1.7976931348623157e308;
    return num / den;
}

__device__ __forceinline__ unsigned long long ballot64(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// diagnostic stamps (separate VO_STAMPS build; never in the product library)
#ifdef VO_STAMPS
#define VO_STAMP(d, slot, idx)                                                                 \
    do {                                                                                       \
        unsigned long long _t;                                                                 \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");            \
        if ((threadIdx.x & 63) == 0 && (d).dbg) (d).dbg[(size_t)(slot) * 16 + (idx)] = _t;   \
    } while (0)
#else
#define VO_STAMP(d, slot, idx) do { } while (0)
#endif
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// ---------------------------------------------------------------------------
// stencil: blur7x7 -> gradients -> 5x5 response -> strict 3x3 NMS candidates
// kernels/feature_extraction_kernel_functions.c:43-120, corner_detection_parallel_GPU.cpp:146-180
//
// Column-streaming form: one wave owns a strip of ST_SW = 114 output columns (two 57-column
// tiles) and walks down a segment of 16 SEGT output rows.  Lane L holds the column PAIR
// c0 = xs - 7 + 2L, c0 + 1 in every stage (128 columns: the strip and 7 halo columns on each
// side; lanes 0..31 hold tile A's columns, lanes 32..63 tile B's).  Vertical neighbours are register histories (one new source row per step);
// horizontal neighbours are the lane's other column or a DPP wave shift (v_mov_b32_dpp
// wave_shr:1 / wave_shl:1), so a shift serves two columns.  No LDS, no barrier.
// Source row k of the segment (y = ys - 7 + k) completes blurred row ys - 10 + k, gradient
// row ys - 11 + k, response row ys - 13 + k and NMS row ys - 14 + k: 14 prologue rows, then
// 16 rows per tile.  Every stage but the response is exact integer arithmetic, so the order
// of its sums is free; the vertical blur runs on both columns at once in 16-bit halves.
// The wave's row and column conditions are uniform branches or lane masks, so the scalar
// unit (one per CU, shared by its four SIMDs) stays well below the VALU's issue rate.
// ---------------------------------------------------------------------------
#define ST_TW VO_TILE_W                // tile width: 57 (56: 12 strips per KITTI row instead of 11; 48: 1080p -3 %)
#define ST_TH VO_TILE_H                // tile height (select reads 16 row counts per tile)
#define ST_SW VO_STRIP_W               // strip width = two tiles: 114 output columns per wave
#ifndef ST_RSEL_ASM
#define ST_RSEL_ASM 1                  // the response's rounding selects ordered by hand (no s_nop)
#endif
#ifndef ST_SOFF_HOIST
#define ST_SOFF_HOIST 1                // a row group's source-row offsets read into SGPRs before its rows
#endif
#ifndef ST_NODOT
#define ST_NODOT 0                     // diagnostic: the horizontal blur without v_dot2_u32_u16
#endif
#ifndef ST_LTMASK_ASM
#define ST_LTMASK_ASM 1                // the NMS maxima's lane masks straight from an asm v_cmp
#endif
#ifndef ST_GRAD_DPP
#define ST_GRAD_DPP (!ST_SHIFT_BPERM)  // the gradients' neighbour columns as DPP operands (not the FLAT form's shifts)
#endif
#ifndef ST_DPP_ADD
#define ST_DPP_ADD 1                   // box sums with v_add_f32_dpp (0: v_mov_b32_dpp + packed adds)
#endif
#ifndef ST_PF_BPERM
#define ST_PF_BPERM 1                  // one-tile-row segments: a row's 128 source bytes by two 64-byte loads and
                                       // two ds_bpermute (instead of two overlapping 128-byte loads)
#endif
#define ST_HALO 7                      // blur 3 + gradient 1 + window 2 + nms 1
#define ST_TCAP VO_TILE_CAP            // candidates per tile (strict maxima: at most one per 2x2 cell)
#ifndef ST_SEGT_DEFAULT
#define ST_SEGT_DEFAULT 6              // tiles per wave segment (VO_STSEG picks 4 / 5 / 6 / 8).  KITTI, alternating runs
                                       // (round 4, gpurun_out r4o): 6 290k, 5 286k, 8 281k, 4 273k -- six-tile segments
                                       // give 44 waves a frame (2.75 workgroups per CU at 64 frames, 8: 33 waves,
                                       // 2.25) at 14 halo rows per 96
#endif
static_assert(ST_SW + 2 * ST_HALO <= 128, "strip + halo within one wave of column pairs");
static_assert(VO_STRIP_XL + ST_TW - 1 == 63, "tile A in lanes 0..31, tile B in lanes 32..63");

#ifndef ST_NOPK
#define ST_NOPK 1                      // k_stencil without packed FP32 (every v_pk_*_f32 split in two v_*_f32):
                                       // the instruction class round 4 saw perturbed next to its MFMA matcher
                                       // (DESIGN.md section 3); four alternating pairs, round 5 (gpurun_out
                                       // r5c_ab): 289.6k with packed FP32, 291.1k without -- within noise, so
                                       // the stencil ships without it (0: the packed form, ST_XSUB_ASM)
#endif
// ST_NOPK: the stencil and every helper it inlines (to the end of k_stencil) compiled without packed
// FP32 -- the whole region, so the kernel's callees keep a subset of its target features and inline
#if ST_NOPK && defined(__HIP_DEVICE_COMPILE__)
#pragma clang attribute push (__attribute__((target("no-packed-fp32-ops"))), apply_to = function)
#endif
// bit casts, popcount and the histogram atomic as the stencil's own inline helpers (the HIP header's
// are defined outside the ST_NOPK region, so a no-packed-FP32 stencil could not inline them)
__device__ __forceinline__ int st_popc(unsigned long long v) { return __builtin_popcountll(v); }
__device__ __forceinline__ int st_f2i(float v) { return __builtin_bit_cast(int, v); }
__device__ __forceinline__ float st_i2f(int v) { return __builtin_bit_cast(float, v); }
__device__ __forceinline__ unsigned st_atomic_add(uint32_t* p, uint32_t v)
{
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int refl101(int i, int n)
{
    if (n == 1) return 0;
    while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
    return i;
}
// DPP wave shifts (gfx9 wave_shr:1 / wave_shl:1): the value of lane L - 1 / lane L + 1.  A DPP
// read of a lane that is off in EXEC returns 0, so the shift must run with the whole wave on:
// the empty volatile asm pins it where it is written (the compiler otherwise sank a shift into
// the masked arm of a select, and border lanes read 0 from their masked neighbours).
#ifndef VO_DPP_PIN
#define VO_DPP_PIN 1
#endif
#ifndef ST_DPP_NOP
#define ST_DPP_NOP 0                   // diagnostic: wait states before every wave shift
#endif
#ifndef ST_SHIFT_BPERM
#define ST_SHIFT_BPERM 0               // diagnostic: wave shifts through ds_bpermute instead of DPP
#endif
__device__ __forceinline__ int shift_bperm(int v, int d)
{
    const int l = (int)(threadIdx.x & 63), src = l + d;
    const int r = __builtin_amdgcn_ds_bpermute(src << 2, v);
    return (src < 0 || src > 63) ? 0 : r;
}
__device__ __forceinline__ int from_left(int v)
{
#if ST_SHIFT_BPERM
    return shift_bperm(v, -1);
#endif
#if ST_DPP_NOP
    asm volatile("s_nop %c1" : "+v"(v) : "i"(ST_DPP_NOP - 1));
#endif
    int r = __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, true);   // bound_ctrl: edge lanes read 0, no old operand
#if VO_DPP_PIN
    asm volatile("" : "+v"(r));
#endif
    return r;
}
__device__ __forceinline__ int from_right(int v)
{
#if ST_SHIFT_BPERM
    return shift_bperm(v, 1);
#endif
#if ST_DPP_NOP
    asm volatile("s_nop %c1" : "+v"(v) : "i"(ST_DPP_NOP - 1));
#endif
    int r = __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, true);   // bound_ctrl: edge lanes read 0, no old operand
#if VO_DPP_PIN
    asm volatile("" : "+v"(r));
#endif
    return r;
}

// XCD-aware workgroup -> (frame, workgroup of the frame) for the extract kernels: a 1-D grid of
// nx * ceil8(nb) workgroups.  Workgroup L is dispatched to XCD L % 8 (round-robin; used for
// speed only, MI355X_MICROARCH.md "Dispatch order ... block->XCD map"), so with d.xcd_map frame z's
// nx workgroups all run on XCD z % 8 and share that XCD's L2: the frame's image and blurred
// plane are fetched into one L2 instead of eight.  false: a padding workgroup of the last group.
__device__ __forceinline__ bool xcd_frame(const VoDev& d, int nx, int nb, int& z, int& bx)
{
    const int L = blockIdx.x;
    if (d.xcd_map) {
        const int k = L >> 3;
        z = (k / nx) * 8 + (L & 7);
        bx = k % nx;
    } else {
        z = L / nx;
        bx = L % nx;
    }
    return z < nb;
}
__host__ inline int xcd_grid(int nx, int nb) { return nx * ((nb + 7) / 8) * 8; }

typedef unsigned short st_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ st_u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(st_u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(st_u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
// wave shifts of 16-bit values (the range lets the blur's products use the 24-bit multiplier)
__device__ __forceinline__ int from_left16(int v)
{
    const int r = from_left(v);
    __builtin_assume((unsigned)r < 65536u);
    return r;
}
__device__ __forceinline__ int from_right16(int v)
{
    const int r = from_right(v);
    __builtin_assume((unsigned)r < 65536u);
    return r;
}
// column pairs in f32 from the blurred plane on: every value up to the response is an integer
// below 2^24 (|J| <= 512 after the blur, a sum of 25 squares < 2^24), so f32 sums are exact and
// their order is free; the pair runs as one packed-FP32 instruction (v_pk_add/mul/fma_f32:
// two lanes' worth per issue, tools/valu_rate.hip)
typedef float st_f2 __attribute__((ext_vector_type(2)));
typedef unsigned short st_w2 __attribute__((ext_vector_type(2)));
// (the box sums add across lanes with hand-written v_add_f32_dpp in k_stencil: the build disables
// LLVM's DPP combine -- it mis-folded a wave shift into v_subrev_u32_dpp on gfx950, Makefile)
__device__ __forceinline__ float from_leftf(float v) { return st_i2f(from_left(st_f2i(v))); }
__device__ __forceinline__ float from_rightf(float v) { return st_i2f(from_right(st_f2i(v))); }
// (a.x - b.y, b.x - a.y) in one v_pk_add_f32: cross halves through op_sel, signs through neg
#ifndef ST_XSUB_ASM
#define ST_XSUB_ASM (!ST_NOPK)         // (the asm form is a v_pk_add_f32)
#endif

__device__ __forceinline__ st_f2 st_xsub(st_f2 a, st_f2 b)
{
#if ST_XSUB_ASM
    st_f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return st_f2{a.x - b.y, b.x - a.y};
#endif
}
__device__ __forceinline__ st_f2 st_fma(st_f2 a, st_f2 b, st_f2 c) { return __builtin_elementwise_fma(a, b, c); }
// the pair's response, kernel .c:108-114 (f32, in the reference's order): det = (jx2 jy2) -
// (sxy sxy); (tr tr) - 4 det as one fma (4 det is exact); (tr * 0.5) - (0.5 * s) == 0.5 * (tr - s)
// exactly (both halvings are exact: tr and s are 0, >= 1 or NaN).  sqrtf correctly rounded for
// this argument, integer-valued (0 or |x| >= 1: every term is an integer-valued f32) or negative
// (NaN): v_sqrt_f32 is within 1 ulp, and one residual test on each neighbour rounds it (the
// compiler's own expansion without its denormal scaling and 0 / inf class test); the two
// residuals of the pair in one packed fma each
__device__ __forceinline__ st_f2 st_response2(st_f2 jx2, st_f2 jy2, st_f2 sxy)
{
    const st_f2 det = (jx2 * jy2) - (sxy * sxy);
    const st_f2 tr = jx2 + jy2;
    const st_f2 x = st_fma(det, st_f2{-4.0f, -4.0f}, tr * tr);
    const st_f2 s = {__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
    const st_f2 sm = {st_i2f(st_f2i(s.x) - 1), st_i2f(st_f2i(s.y) - 1)};
    const st_f2 sp = {st_i2f(st_f2i(s.x) + 1), st_i2f(st_f2i(s.y) + 1)};
    const st_f2 rm = st_fma(-sm, s, x), rp = st_fma(-sp, s, x);
    st_f2 r;
#if ST_RSEL_ASM
    // r = rp > 0 ? sp : (rm <= 0 ? sm : s) per component (NaN: s), the four compares into SGPR
    // pairs first, so every select reads a mask written two or more instructions earlier (left to
    // itself LLVM pairs each compare with its select through VCC and pads it with s_nop 1)
    {
        unsigned long long ma, mb, mc, md;
        float tx, ty;
        asm(
            "v_cmp_ge_f32_e64 %[mc], 0, %[rmx]\n\t"
            "v_cmp_ge_f32_e64 %[md], 0, %[rmy]\n\t"
            "v_cmp_lt_f32_e64 %[ma], 0, %[rpx]\n\t"
            "v_cmp_lt_f32_e64 %[mb], 0, %[rpy]\n\t"
            "v_cndmask_b32_e64 %[tx], %[sx], %[smx], %[mc]\n\t"
            "v_cndmask_b32_e64 %[ty], %[sy], %[smy], %[md]\n\t"
            "v_cndmask_b32_e64 %[rx], %[tx], %[spx], %[ma]\n\t"
            "v_cndmask_b32_e64 %[ry], %[ty], %[spy], %[mb]"
            : [ma] "=&s"(ma), [mb] "=&s"(mb), [mc] "=&s"(mc), [md] "=&s"(md), [tx] "=&v"(tx), [ty] "=&v"(ty),
              [rx] "=&v"(r.x), [ry] "=&v"(r.y)
            : [rmx] "v"(rm.x), [rmy] "v"(rm.y), [rpx] "v"(rp.x), [rpy] "v"(rp.y), [sx] "v"(s.x), [sy] "v"(s.y),
              [smx] "v"(sm.x), [smy] "v"(sm.y), [spx] "v"(sp.x), [spy] "v"(sp.y));
    }
#else
    r.x = rp.x > 0.0f ? sp.x : (rm.x <= 0.0f ? sm.x : s.x);
    r.y = rp.y > 0.0f ? sp.y : (rm.y <= 0.0f ? sm.y : s.y);
#endif
#if VO_RESP_SCALE == 2
    return tr - r;                    // twice the response (exact): see VO_RESP_SCALE
#else
    return 0.5f * (tr - r);
#endif
}
// f(integral_constant<int, I>) for I = 0 .. N-1, unrolled at compile time
template <typename F, int... I>
__device__ __forceinline__ void st_for(F&& f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}
#define ST_BUF_DW3 0x00020000
#ifndef ST_FLAT_DEFAULT
#define ST_FLAT_DEFAULT 0     // VO_ST_FLAT=1: the branch-free FLAT form where the margins allow it (measured slower:
                              // KITTI 264k vs 283k frames/s, stencil 2.01 vs 1.81 us/frame; parity-tested as a knob)
#endif
#ifndef LDS_POISON
#define LDS_POISON 0      // diagnostic build: k_select / k_describe poison their LDS first
#endif
#ifndef ST_DROP_SOFFSET
#define ST_DROP_SOFFSET 0
#endif      // gfx9 buffer descriptor word 3 (raw bytes, no format)

#ifndef SL_STAGE2
#define SL_STAGE2 1                    // k_select: two threads per tile stage its keys (eight loads in flight)
#endif
#ifndef ST_LHIST
#define ST_LHIST 1                     // k_select builds the histogram from its keys; the stencil writes none
#endif
// WRITE_SIZE attribution probes (diagnostic builds only, tools/stencil_write_probe.py): the stencil
// without its blurred-plane stores (1), its key and tile-row stores (2), its histogram atomics (4)
#ifndef ST_PROBE_NOSTORE
#define ST_PROBE_NOSTORE 0
#endif
#ifndef ST_HIST_FLUSH
#define ST_HIST_FLUSH 0   // the general form's histogram counts at the group flush (from the LDS keys)
#endif
#ifndef ST_KEYS_LDS
#define ST_KEYS_LDS 1     // the general form stages a tile pair's keys in LDS and writes them once per
                          // 16-row group, contiguously (0: a divergent 8-byte global store per maximum)
#endif
// grid xcd_grid(ceil(waves / 4), nb): 4 waves per workgroup, one (strip, segment) per wave
#ifndef ST_WAVES_PER_EU
#define ST_WAVES_PER_EU 4
#endif
// FLAT (launch_stencil: NMS margins of 5+ rows and columns, no response map): the image's border
// rows and columns cannot reach a maximum inside the margins (a response at row y needs gradient
// rows y - 2 .. y + 2, an NMS centre at row >= 5 has neighbours at rows >= 4: gradient rows >= 2,
// and likewise at the bottom and the sides), so their gradient masks are dropped; the candidate
// keys and histogram counts are stored through buffer descriptors whose out-of-range offset drops
// the lanes that hold no maximum (tests/test_buffer_range.py).  A 16-row group is then one basic
// block with no branch, and the scheduler overlaps consecutive rows' dependency chains.
// NH: no histogram -- the batch's select is the one-workgroup k_select, which builds the histogram
// in LDS from the keys it stages (the stencil's agent-scope histogram atomics go to memory: 232 KB of
// WRITE per KITTI frame against a 16 KB histogram, tools/stencil_write_probe.py, r6c)
template <int SEGT, bool DBG, bool FLAT, bool NH = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ST_WAVES_PER_EU))) k_stencil(VoDev d, const uint8_t* __restrict__ img0, size_t frame_bytes,
                                                  int write_response, int nb)
{
    constexpr int SEG = ST_TH * SEGT;
    const int W = d.W, H = d.H;
    const int ntx = (W + ST_TW - 1) / ST_TW, nsx = (ntx + 1) / 2, nty = (H + ST_TH - 1) / ST_TH;
    const int nseg = (nty + SEGT - 1) / SEGT;
    // frame z of the batch (its image and its scratch copy), workgroup bx of the frame
    int z, bx;
    if (!xcd_frame(d, (nsx * nseg + 3) / 4, nb, z, bx)) return;
    const int g = bx * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
    if (g >= nsx * nseg) return;
    const int sxi = g % nsx, seg = g / nsx;
    const int lane = threadIdx.x & 63;
#if ST_KEYS_LDS
    // this wave's tile pair's keys (+ 128 lane-private slots: the FLAT form's lanes without a maximum)
    __shared__ uint64_t s_keys[4][2 * ST_TCAP + (FLAT ? 128 : 0)];
    uint64_t* __restrict__ wkeys = s_keys[threadIdx.x >> 6];
#endif
    // image rows and blurred rows through buffer descriptors: the row offset is a scalar
    // operand of the access (no per-row address arithmetic), and a lane whose offset is past
    // the plane (the halo lanes' stores) is dropped by the range check
    const __amdgpu_buffer_rsrc_t rimg =
        __builtin_amdgcn_make_buffer_rsrc((void*)(img0 + (size_t)z * frame_bytes), 0, W * H, ST_BUF_DW3);
    const __amdgpu_buffer_rsrc_t rblur =
        __builtin_amdgcn_make_buffer_rsrc((void*)(d.blurred + (size_t)z * d.bplane), 0, (int)d.bplane, ST_BUF_DW3);
    uint64_t* __restrict__ cand = d.cand + (size_t)z * d.cand_cap;
    uint8_t* __restrict__ tilerows = d.tilerows + (size_t)z * d.ntiles * ST_TH;
    uint32_t* __restrict__ hist = d.hist + (size_t)z * VO_HIST_BINS;
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t rcand =
        __builtin_amdgcn_make_buffer_rsrc((void*)cand, 0, (int)(d.cand_cap * 8u), ST_BUF_DW3);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t rhist =
        __builtin_amdgcn_make_buffer_rsrc((void*)hist, 0, VO_HIST_BINS * 4, ST_BUF_DW3);
    const int Wb = d.bstride;
    // wave shifts: pinned against sinking into a masked arm, except in the FLAT form (no masked arm)
    auto shl = [](int v) { if constexpr (FLAT && !ST_SHIFT_BPERM) return __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, true); else return from_right(v); };
    auto shr = [](int v) { if constexpr (FLAT && !ST_SHIFT_BPERM) return __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, true); else return from_left(v); };
    [[maybe_unused]] auto shrf = [&](float v) { return st_i2f(shr(st_f2i(v))); };
    [[maybe_unused]] auto shlf = [&](float v) { return st_i2f(shl(st_f2i(v))); };

    const int xs = sxi * ST_SW, ys = seg * SEG;
    const int c0 = xs - VO_STRIP_XL + 2 * lane;                // this lane's columns: c0, c0 + 1
    const int xl0 = refl101(c0, W), xl1 = refl101(c0 + 1, W);  // BORDER_REFLECT_101
    auto outc = [&](int x) { return x >= xs && x < xs + ST_SW; };   // the strip's output columns
    // blurred store (bytes c0, c0 + 1 at plane offset c0 + VO_BLUR_X0: 2-byte aligned): out of
    // range for pairs off the strip and past the image's last column.  A pair half off the strip
    // stores its neighbour strip's column too -- the same value that strip's wave stores.
    const int boff = (outc(c0) || outc(c0 + 1)) && c0 < W ? c0 + VO_BLUR_X0 : 0x40000000;
    int boffq = boff;                  // the voffset of a group's last 4 rows (set per group below)
    const bool isB = lane >= 32;                              // the strip's second tile
    const bool hasB = 2 * sxi + 1 < ntx;
    // the wave's columns reach the image's outer two columns, where gradients (kernel .c:59-76)
    // are 0: the lane masks apply only then
    const bool colfix = xs - VO_STRIP_XL < 2 || xs - VO_STRIP_XL + 128 > W - 2;
    const bool g0 = c0 >= 1 && c0 <= W - 2, g1 = c0 + 1 >= 1 && c0 + 1 <= W - 2;
    // lane masks folded into lane constants, so a row's tests are one compare each: responses
    // outside 2 <= j <= W-3 are 0 (kernel .c:97-114): their threshold is +inf; an NMS centre
    // outside the margin meets a neighbour maximum of INT_MAX
    const float thr = d.resp_thr;
    const float thr0 = c0 >= 2 && c0 <= W - 3 ? thr : __builtin_inff();
    const float thr1 = c0 + 1 >= 2 && c0 + 1 <= W - 3 ? thr : __builtin_inff();
    const int hk = d.nms_k / 2;
    auto ncol = [&](int x) { return outc(x) && x >= hk && x < W - hk && x >= d.bcol && x <= W - d.bcol; };
    const int nmsk0 = ncol(c0) ? 0 : 0x7FFFFFFF, nmsk1 = ncol(c0 + 1) ? 0 : 0x7FFFFFFF;
    const int nlo = max(hk, d.brow), nhi = max(nlo, min(H - hk, H - d.brow + 1));   // NMS rows [nlo, nhi)
    const uint32_t thr_bits = d.thr_bits;
    // (halo columns are never maxima: their NMS masks, so a tile's lane masks are halves of the wave)
    constexpr unsigned long long mA = 0xFFFFFFFFull;          // lanes 0 .. 31: tile 2 sxi
    constexpr unsigned long long mB = mA << 32;               // lanes 32 .. 63: tile 2 sxi + 1

    // register histories (index 0 oldest); source rows packed: column c0 low half, c0 + 1 high
    uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0, s6 = 0;
    const st_f2 z2 = {0.0f, 0.0f};
    st_f2 BA = z2, BM = z2, BE = z2;                                          // blurred rows
    st_f2 QX[5] = {z2, z2, z2, z2, z2}, VX = z2;                              // Jx^2 rows, vertical sums
    st_f2 QY[5] = {z2, z2, z2, z2, z2}, VY = z2;                              // Jy^2
    st_f2 QS[5] = {z2, z2, z2, z2, z2}, VS = z2;                              // Jxy
    int ru0 = 0, rm0 = 0, rd0 = 0, ru1 = 0, rm1 = 0, rd1 = 0;               // response rows (f32 bits)
    int toffA = 0, toffB = 0;                                                // candidates so far per tile
    int trows = 0;                                                           // lane r (16 + r): tile A (B) row r count
#if ST_DIAG & 2
    unsigned long long dck = 0ull;                                           // checksum of the keys this lane stored
    unsigned long long sck = 0ull, rck = 0ull;                               // source rows consumed, responses computed
    const int dfr = d.diag_f0 + z;                                           // frame index (diagnostic arrays)
#elif ST_DIAG & 4
    uint32_t lsck = 0u;                                                      // light: source rows consumed (one mad a row)
    const int dfr = d.diag_f0 + z;
#endif

    // lane u of the result: byte offset of source row ys - 7 + k0 + u (u < 16)
    auto row_offsets = [&](int k0) {
        const int y = refl101(ys - ST_HALO + k0 + (lane & 15), H);
        return y * W;                                          // frames < 2^31 px
    };
#if ST_PF_BPERM
    constexpr bool BP = SEGT == 1;
#else
    constexpr bool BP = false;
#endif
    // BP: lane l loads window columns l and 64 + l (one 64-byte span per load), packed as bytes 0 / 1;
    // its pair (window columns 2l, 2l + 1) comes back by two ds_bpermute and a byte select
    const int xa = refl101(xs - VO_STRIP_XL + lane, W), xb = refl101(xs - VO_STRIP_XL + 64 + lane, W);
    const int bpi0 = ((2 * lane) & 63) << 2, bpi1 = ((2 * lane + 1) & 63) << 2;
    const uint32_t bsel = lane >= 32 ? 0x0c050c01u : 0x0c040c00u;
    auto unpack = [&](uint32_t P) -> uint32_t {
        if constexpr (BP) {
            const uint32_t r0 = (uint32_t)__builtin_amdgcn_ds_bpermute(bpi0, (int)P);
            const uint32_t r1 = (uint32_t)__builtin_amdgcn_ds_bpermute(bpi1, (int)P);
            return __builtin_amdgcn_perm(r1, r0, bsel);
        } else {
            return P;
        }
    };
    auto load = [&](int soff) -> uint32_t {
        if constexpr (BP) {
            const uint32_t a = __builtin_amdgcn_raw_buffer_load_b8(rimg, xa, soff, 0);
            const uint32_t b = __builtin_amdgcn_raw_buffer_load_b8(rimg, xb, soff, 0);
            return a | (b << 8);
        }
        const uint32_t a = __builtin_amdgcn_raw_buffer_load_b8(rimg, xl0, soff, 0);
        const uint32_t b = __builtin_amdgcn_raw_buffer_load_b8(rimg, xl1, soff, 0);
        return a | (b << 16);
    };

    // one source row through every stage that is live at step k (P: 1 blur, 2 + gradients,
    // 3 + blurred store, 4 + response, 5 + NMS of tile row R)
    auto step = [&](auto PH, int k, uint32_t src, auto R) {
        constexpr int P = decltype(PH)::value;
        constexpr int r = decltype(R)::value;
        s0 = s1; s1 = s2; s2 = s3; s3 = s4; s4 = s5; s5 = s6; s6 = src;
#if ST_DIAG & 2
        sck += mix64((uint64_t)src ^ ((uint64_t)(uint32_t)k << 32));
#elif ST_DIAG & 4
        lsck = lsck * 0x01000193u + src;
#endif
        if constexpr (P >= 1) {
            // 1. 7x7 blur (cv::GaussianBlur 8U fixed point, A.1): vertical taps on both columns
            //    in 16-bit halves (<= 65280); the horizontal taps as dot products of 16-bit pairs
            //    (v_dot2_u32_u16) of the lane's pair and its neighbours' (wave shifts of the packed
            //    word move both columns), the rounding bias as the first addend:
            //    (sum k_i k_j I + 2^15) >> 16 is byte 2 of the sum (< 2^24)
            const st_u16x2 v = (as_u16x2(s0) + as_u16x2(s6)) * (unsigned short)8 +
                               (as_u16x2(s1) + as_u16x2(s5)) * (unsigned short)28 +
                               (as_u16x2(s2) + as_u16x2(s4)) * (unsigned short)56 + as_u16x2(s3) * (unsigned short)72;
            const uint32_t V = as_u32(v);
            const uint32_t VL = (uint32_t)shr((int)V), VR = (uint32_t)shl((int)V);
            const uint32_t VL2 = (uint32_t)shr((int)VL), VR2 = (uint32_t)shl((int)VR);
#if ST_NODOT
            auto dot = [](uint32_t a, st_w2 w, uint32_t c) { return (a & 0xFFFFu) * (uint32_t)w.x + (a >> 16) * (uint32_t)w.y + c; };
#else
            auto dot = [](uint32_t a, st_w2 w, uint32_t c) { return __builtin_amdgcn_udot2(as_u16x2(a), w, c, false); };
#endif
            // column c0: 72 I(c0) + 56 (I(c0-1) + I(c0+1)) + 28 (I(c0-2) + I(c0+2)) + 8 (I(c0-3) + I(c0+3))
            const uint32_t ha = dot(VR, st_w2{28, 8}, dot(VL2, st_w2{0, 8}, dot(VL, st_w2{28, 56}, dot(V, st_w2{72, 56}, 32768u))));
            const uint32_t hb = dot(VR2, st_w2{8, 0}, dot(VR, st_w2{56, 28}, dot(VL, st_w2{8, 28}, dot(V, st_w2{56, 72}, 32768u))));
            BA = BM; BM = BE;
            BE = st_f2{(float)((ha >> 16) & 255u), (float)((hb >> 16) & 255u)};
            if constexpr (P >= 3) {
                // blurred row ys - 10 + k: the plane is padded to whole strips and 4 rows past the
                // last tile, so every output lane stores; rows past the segment (k >= SEG + 10:
                // the last 4 rows of the segment's last tile row group) are the next segment's
                // (the same values, stored by its wave), so their store is dropped by an
                // out-of-range *voffset* (boffq).  gfx950's raw-buffer range check covers voffset +
                // soffset (tests/hip/buffer_range_probe.hip, tests/test_buffer_range.py: a
                // straddling store keeps its in-range lanes, nothing lands past num_records), so
                // round 3's drop through soffset was also safe; voffset keeps the row offset in
                // soffset a plain scalar operand.
#if ST_DROP_SOFFSET
                // round 3's form, kept for the A/B evidence run only (tools/gpu_det.sh): the drop in soffset
                const int brow = k < SEG + 10 ? (ys - 10 + k) * Wb : 0x40000000;
                __builtin_amdgcn_raw_buffer_store_b16((unsigned short)__builtin_amdgcn_perm(hb, ha, 0x0c0c0602u), rblur, boff,
                                                      brow, 0);
                (void)boffq;
#else
                if constexpr (ST_PROBE_NOSTORE & 1) {
                } else if constexpr (P == 5 && r >= ST_TH - 4) {
                    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)__builtin_amdgcn_perm(hb, ha, 0x0c0c0602u), rblur,
                                                          boffq, (ys - 10 + k) * Wb, 0);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)__builtin_amdgcn_perm(hb, ha, 0x0c0c0602u), rblur,
                                                          boff, (ys - 10 + k) * Wb, 0);
                }
#endif
            }
        }
        if constexpr (P >= 2) {
            // 2. gradients of row yg (kernel .c:59-76), 0 outside 1 <= i <= H-2, 1 <= j <= W-2;
            //    the reference's f32 values are these integers (all below 2^11)
            const int yg = ys - 11 + k;
            const st_f2 DV = BA - BE, SV = st_fma(BM, st_f2{2.0f, 2.0f}, BA + BE);
#if ST_GRAD_DPP
            // the neighbour columns' dv / sv as DPP operands of the adds and subtracts that use them
            // (the same operations on the same values as the shifted-copy form below: six VALU for
            // its four v_mov_b32_dpp and six adds / subtracts).  s_nop 1: the two wait states a DPP
            // read of a VGPR written by the previous VALU needs (DV and SV are computed just before)
            float a1, a2, jy0, jy1, jxy0, jxy1;
            asm("s_nop 1\n\t"
                "v_add_f32_dpp %[a1], %[dy], %[dy] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                "v_add_f32_dpp %[a2], %[dx], %[dx] wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                "v_sub_f32_dpp %[jxy0], %[dy], %[dy] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                "v_subrev_f32_dpp %[jxy1], %[dx], %[dx] wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                "v_sub_f32_dpp %[jy0], %[sy], %[sy] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                "v_subrev_f32_dpp %[jy1], %[sx], %[sx] wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
                : [a1] "=&v"(a1), [a2] "=&v"(a2), [jxy0] "=&v"(jxy0), [jxy1] "=&v"(jxy1), [jy0] "=&v"(jy0),
                  [jy1] "=&v"(jy1)
                : [dx] "v"(DV.x), [dy] "v"(DV.y), [sx] "v"(SV.x), [sy] "v"(SV.y));
            st_f2 JX = st_fma(DV, st_f2{2.0f, 2.0f}, st_f2{a1, a2}); // (dL + 2 dv0 + dv1, dv0 + 2 dv1 + dR)
            st_f2 JY = {jy0, jy1};                                    // (sL - sv1, sv0 - sR)
            st_f2 JXY = {jxy0, jxy1};                                 // (dL - dv1, dv0 - dR)
#else
            const st_f2 Y = {shrf(DV.y), shlf(DV.x)};                 // dv of columns c0 - 1, c0 + 2
            const st_f2 Z = {shrf(SV.y), shlf(SV.x)};
            st_f2 JX = st_fma(DV, st_f2{2.0f, 2.0f}, Y + DV.yx);      // (dL + 2 dv0 + dv1, dv0 + 2 dv1 + dR)
            st_f2 JY = st_xsub(Z, SV);                                // (sL - sv1, sv0 - sR)
            st_f2 JXY = st_xsub(Y, DV);                               // (dL - dv1, dv0 - dR)
#endif
            // both conditions are wave-uniform and rare (the image's outer columns and rows): the
            // empty volatile asm keeps them branches (if-converted, they cost 12 selects a row)
            if constexpr (!FLAT) {
                if (colfix) {
                    asm volatile("");
                    if (!g0) JX.x = JY.x = JXY.x = 0.0f;
                    if (!g1) JX.y = JY.y = JXY.y = 0.0f;
                }
                if ((unsigned)(yg - 1) > (unsigned)(H - 3)) {
                    asm volatile("");
                    JX = JY = JXY = z2;
                }
            }
            // 3. 5x5 window sums (kernel .c:97-107): vertical running sums, then horizontal
            const st_f2 X2 = JX * JX, Y2 = JY * JY;
            VX = VX + (X2 - QX[0]); VY = VY + (Y2 - QY[0]); VS = VS + (JXY - QS[0]);
#pragma unroll
            for (int i = 0; i < 4; ++i) { QX[i] = QX[i + 1]; QY[i] = QY[i + 1]; QS[i] = QS[i + 1]; }
            QX[4] = X2; QY[4] = Y2; QS[4] = JXY;
        }
        if constexpr (P >= 4) {
            // horizontal 5-sums: column c0 takes c0-2 .. c0+2 = the left pair, its own pair and
            // the right lane's c0; column c0 + 1 the left lane's c0 + 1, its pair, the right pair
#if ST_DPP_ADD
            // (exact integer sums below 2^24: the order is free) per plane four DPP adds and one add,
            // the three planes in one block ordered so that every DPP source was written at least
            // two VALU instructions earlier (the wait states a DPP read of a fresh VGPR needs; the
            // inputs come from before the block): no s_nop
            float sx0, sx1, sy0, sy1, ss0, ss1;
            {
                float pX, pY, pS, xX, yX, xY, yY, xS, yS;
                asm(
#if ST_DPP_NOP
                    "s_nop 7\n\t"
#endif
                    "v_add_f32 %[pX], %[ax], %[ay]\n\t"
                    "v_add_f32 %[pY], %[bx], %[by]\n\t"
                    "v_add_f32 %[pS], %[cx], %[cy]\n\t"
                    "v_add_f32_dpp %[xX], %[pX], %[pX] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                    "v_add_f32_dpp %[yX], %[ay], %[pX] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                    "v_add_f32_dpp %[xY], %[pY], %[pY] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                    "v_add_f32_dpp %[yY], %[by], %[pY] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                    "v_add_f32_dpp %[xS], %[pS], %[pS] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                    "v_add_f32_dpp %[yS], %[cy], %[pS] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                    "v_add_f32_dpp %[sx0], %[ax], %[xX] wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                    "v_add_f32_dpp %[sx1], %[pX], %[yX] wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                    "v_add_f32_dpp %[sy0], %[bx], %[xY] wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                    "v_add_f32_dpp %[sy1], %[pY], %[yY] wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                    "v_add_f32_dpp %[ss0], %[cx], %[xS] wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
                    "v_add_f32_dpp %[ss1], %[pS], %[yS] wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
                    : [pX] "=&v"(pX), [pY] "=&v"(pY), [pS] "=&v"(pS), [xX] "=&v"(xX), [yX] "=&v"(yX),
                      [xY] "=&v"(xY), [yY] "=&v"(yY), [xS] "=&v"(xS), [yS] "=&v"(yS),
                      [sx0] "=&v"(sx0), [sx1] "=&v"(sx1), [sy0] "=&v"(sy0), [sy1] "=&v"(sy1),
                      [ss0] "=&v"(ss0), [ss1] "=&v"(ss1)
                    : [ax] "v"(VX.x), [ay] "v"(VX.y), [bx] "v"(VY.x), [by] "v"(VY.y), [cx] "v"(VS.x), [cy] "v"(VS.y));
            }
            const st_f2 SX = {sx0, sx1}, SY = {sy0, sy1}, SS = {ss0, ss1};
#else
            auto box = [](st_f2 a) {
                const st_f2 p = a + a.yx;                              // (a0 + a1, a0 + a1)
                const st_f2 l = {from_leftf(p.x), from_leftf(a.y)};
                const st_f2 r = {from_rightf(a.x), from_rightf(p.x)};
                return (l + p) + r;
            };
            const st_f2 SX = box(VX), SY = box(VY), SS = box(VS);
#endif
            // 4. response of row yr (kernel .c:108-114), 0 outside 2 <= i <= H-3, 2 <= j <= W-3
            const int yr = ys - 13 + k;
            const bool rrow = (unsigned)(yr - 2) <= (unsigned)(H - 5);
            const st_f2 rv = st_response2(SX, SY, SS);
            const int o0 = ((rv.x > thr0) & rrow) ? st_f2i(rv.x) : 0;
            const int o1 = ((rv.y > thr1) & rrow) ? st_f2i(rv.y) : 0;
            if constexpr (DBG) {
                if (write_response && yr >= ys && yr < min(ys + SEG, H)) {
                    float* R = d.response + (size_t)yr * W;
                    const float w0 = write_response == 2 ? SX.x : write_response == 3 ? SY.x
                                   : write_response == 4 ? SS.x : st_i2f(o0) * (1.0f / VO_RESP_SCALE);
                    const float w1 = write_response == 2 ? SX.y : write_response == 3 ? SY.y
                                   : write_response == 4 ? SS.y : st_i2f(o1) * (1.0f / VO_RESP_SCALE);
                    if (outc(c0) && c0 >= 0 && c0 < W) R[c0] = w0;
                    if (outc(c0 + 1) && c0 + 1 < W) R[c0 + 1] = w1;
                }
            }
            ru0 = rm0; rm0 = rd0; rd0 = o0;
            ru1 = rm1; rm1 = rd1; rd1 = o1;
#if ST_DIAG & 2
            rck += mix64((((uint64_t)(uint32_t)o0 << 32) | (uint32_t)o1) ^ ((uint64_t)(uint32_t)k << 48));
#endif
        }
        if constexpr (P >= 5) {
            // 5. strict 3x3 NMS of row yn = tile row r inside the retinal margin
            //    (corner_detection_parallel_GPU.cpp:152-180): any neighbour >= the centre rejects
            //    it; responses are +0 or above resp_thr >= 0 (vo_create), so their bit patterns
            //    order as the values do and the window maximum is an integer max3
            const int yn = ys - 14 + k;
            const int cm0 = max(max(ru0, rm0), rd0), cm1 = max(max(ru1, rm1), rd1);
            const int cL = shr(cm1), cR = shl(cm0);
            const int nb0 = max(max(cL, cm1), max(max(ru0, rd0), nmsk0));
            const int nb1 = max(max(cm0, cR), max(max(ru1, rd1), nmsk1));
            const bool rok = (unsigned)(yn - nlo) < (unsigned)(nhi - nlo);
            // the maxima's lane masks straight from the compares (a ballot of a compare ANDed with
            // rok materialised the lane bools and compared them again, 4 VALU a row); rok is
            // wave-uniform and masks them as scalars, and inside the branch it holds
            auto lt_mask = [](int a, int b) {
#if ST_LTMASK_ASM
                unsigned long long m;
                asm("v_cmp_lt_i32_e64 %0, %1, %2" : "=s"(m) : "v"(a), "v"(b));
                return m;
#else
                return (unsigned long long)__builtin_amdgcn_ballot_w64(a < b);
#endif
            };
            const unsigned long long rokm = rok ? ~0ull : 0ull;      // (a select, not a branch around the compare)
            const unsigned long long b0 = lt_mask(nb0, rm0) & rokm, b1 = lt_mask(nb1, rm1) & rokm;
            // (rok: the NMS rows; the general form reaches the stores only through b0 | b1, which rok masks)
            const bool mx0 = rok && nb0 < rm0, mx1 = rok && nb1 < rm1;
            const int cA = st_popc(b0 & mA) + st_popc(b1 & mA);
            const int cB = st_popc(b0 & mB) + st_popc(b1 & mB);
            // (readfirstlane: the counts are wave-uniform SGPR values already -- a no-op -- but the
            // ST_NOPK build's compiler keeps them in VGPRs without it)
            asm("v_writelane_b32 %0, %1, %2" : "+v"(trows) : "s"(__builtin_amdgcn_readfirstlane(cA)), "n"(r));
            asm("v_writelane_b32 %0, %1, %2" : "+v"(trows) : "s"(__builtin_amdgcn_readfirstlane(cB)), "n"(16 + r));
            if constexpr (FLAT) {
                const uint32_t pos0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32),
                                      __builtin_amdgcn_mbcnt_lo((uint32_t)b1,
                                      __builtin_amdgcn_mbcnt_hi((uint32_t)(b0 >> 32),
                                      __builtin_amdgcn_mbcnt_lo((uint32_t)b0, 0u))));
                const uint32_t base = (uint32_t)(isB ? ST_TCAP + toffB - cA : toffA) + pos0;
                const uint32_t key_lo = ((uint32_t)yn << 16) | (uint32_t)c0;
#if ST_KEYS_LDS
                // every lane writes LDS: a lane without a maximum into its own slot past the pair's
                // (the histogram counts follow from the flushed keys, once per 16-row group)
                const int s0 = mx0 ? (int)base : 2 * ST_TCAP + lane;
                const int s1 = mx1 ? (int)(base + (mx0 ? 1u : 0u)) : 2 * ST_TCAP + 64 + lane;
                wkeys[s0] = ((uint64_t)(uint32_t)rm0 << 32) | key_lo;
                wkeys[s1] = ((uint64_t)(uint32_t)rm1 << 32) | (key_lo + 1u);
#else
                // every lane stores; a lane without a maximum gets an out-of-range offset (dropped)
                const uint32_t slot0 = (uint32_t)((yn / ST_TH) * ntx + 2 * sxi) * ST_TCAP + base;
                const int o0 = mx0 ? (int)(slot0 * 8u) : 0x7FFFFFF0;
                const int o1 = mx1 ? (int)((slot0 + (mx0 ? 1u : 0u)) * 8u) : 0x7FFFFFF0;
                typedef unsigned int st_u2 __attribute__((ext_vector_type(2)));
                __builtin_amdgcn_raw_buffer_store_b64(st_u2{key_lo, (uint32_t)rm0}, rcand, o0, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b64(st_u2{key_lo + 1u, (uint32_t)rm1}, rcand, o1, 0, 0);
                const int h0 = mx0 ? (int)(min(((uint32_t)rm0 - thr_bits) >> 15, (uint32_t)(VO_HIST_BINS - 1)) * 4u) : 0x7FFFFFF0;
                const int h1 = mx1 ? (int)(min(((uint32_t)rm1 - thr_bits) >> 15, (uint32_t)(VO_HIST_BINS - 1)) * 4u) : 0x7FFFFFF0;
                if constexpr (!NH) {
                    (void)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, rhist, h0, 0, 0);
                    (void)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, rhist, h1, 0, 0);
                }
#endif
            } else if (b0 | b1) {
                // tile-local raster order: rows before this one, then columns before: the lower
                // lanes' pairs, and c0 before c0 + 1
                const uint32_t pos0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32),
                                      __builtin_amdgcn_mbcnt_lo((uint32_t)b1,
                                      __builtin_amdgcn_mbcnt_hi((uint32_t)(b0 >> 32),
                                      __builtin_amdgcn_mbcnt_lo((uint32_t)b0, 0u))));
                const uint32_t base = (uint32_t)(isB ? ST_TCAP + toffB - cA : toffA) + pos0;
                const uint32_t key_lo = ((uint32_t)yn << 16) | (uint32_t)c0;
#if ST_KEYS_LDS
                uint64_t* __restrict__ tk = wkeys;
#else
                const int tileA = (yn / ST_TH) * ntx + 2 * sxi;
                uint64_t* __restrict__ tk = cand + (size_t)tileA * ST_TCAP;
#endif
                if (mx0) {
                    tk[base] = ((uint64_t)(uint32_t)rm0 << 32) | key_lo;
#if !(ST_KEYS_LDS && ST_HIST_FLUSH)
                    const uint32_t bin = min(((uint32_t)rm0 - thr_bits) >> 15, (uint32_t)(VO_HIST_BINS - 1));
                    if (!(ST_PROBE_NOSTORE & 4) && !NH) st_atomic_add(&hist[bin], 1u);
#endif
#if ST_DIAG & 2
                    dck += mix64((((uint64_t)(uint32_t)rm0 << 32) | key_lo) ^ ((uint64_t)base << 48));
#endif
                }
                if (mx1) {
                    tk[base + (mx0 ? 1u : 0u)] = ((uint64_t)(uint32_t)rm1 << 32) | (key_lo + 1u);
#if !(ST_KEYS_LDS && ST_HIST_FLUSH)
                    const uint32_t bin = min(((uint32_t)rm1 - thr_bits) >> 15, (uint32_t)(VO_HIST_BINS - 1));
                    if (!(ST_PROBE_NOSTORE & 4) && !NH) st_atomic_add(&hist[bin], 1u);
#endif
#if ST_DIAG & 2
                    dck += mix64((((uint64_t)(uint32_t)rm1 << 32) | (key_lo + 1u)) ^ ((uint64_t)(base + (mx0 ? 1u : 0u)) << 48));
#endif
                }
            }
            toffA += cA; toffB += cB;
        }
    };
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    using P2 = std::integral_constant<int, 2>;
    using P3 = std::integral_constant<int, 3>;
    using P4 = std::integral_constant<int, 4>;
    using P5 = std::integral_constant<int, 5>;
    using R0 = std::integral_constant<int, 0>;

    // prologue: source rows ys-7 .. ys+6 (blurred rows from ys-4, gradients from ys-3,
    // responses from ys-1: what the segment's first NMS row needs); then the first 8 rows of
    // the main loop are requested
    // source rows in flight ahead of the step: 8; 16 in the one-tile-row segments of the per-frame
    // call, so that its whole 30-row walk is requested up front (it reads the frame from pinned host
    // memory: a second wave of requests paid the PCIe latency again)
    constexpr int LA = SEGT == 1 ? 16 : 8;
    uint32_t ahead[LA];
    {
        const int rows = row_offsets(0);
        uint32_t src[14];
        st_for([&](auto U) { src[U] = load(__builtin_amdgcn_readlane(rows, U)); }, std::make_integer_sequence<int, 14>{});
        const int rows2 = row_offsets(14);
        st_for([&](auto U) { ahead[U] = load(__builtin_amdgcn_readlane(rows2, U)); }, std::make_integer_sequence<int, LA>{});
        if constexpr (BP) st_for([&](auto U) { src[U] = unpack(src[U]); }, std::make_integer_sequence<int, 14>{});
        st_for([&](auto U) { step(P0{}, U, src[U], R0{}); }, std::make_integer_sequence<int, 6>{});
        step(P1{}, 6, src[6], R0{});
        step(P1{}, 7, src[7], R0{});
        step(P2{}, 8, src[8], R0{});
        step(P2{}, 9, src[9], R0{});
        step(P3{}, 10, src[10], R0{});
        step(P3{}, 11, src[11], R0{});
        step(P4{}, 12, src[12], R0{});
        step(P4{}, 13, src[13], R0{});
    }
    // BP: row k0 + U's pair unpacked one row ahead of its step (the ds_bpermute latency under the step)
    uint32_t nxt = BP ? unpack(ahead[0]) : 0u;
    // one tile row group (16 rows) per iteration; the last segment may hold fewer tiles.  Row
    // k0 + u + LA is requested as row k0 + u is consumed (the last group's requests past the
    // segment read rows that are never used)
    const int ntl = min(SEGT, nty - seg * SEGT);
    for (int i = 0; i < ntl; ++i) {
        const int k0 = 14 + ST_TH * i;
        const int rows = row_offsets(k0 + LA);
        toffA = 0; toffB = 0;
        // rows k0 + 12 .. k0 + 15 reach past the segment (k >= SEG + 10) only in its last group
        static_assert(14 + ST_TH * (SEGT - 1) + (ST_TH - 4) == SEG + 10, "segment tail rows");
        boffq = i == SEGT - 1 ? 0x40000000 : boff;
        // the group's 16 row offsets to SGPRs up front: a v_readlane right before the buffer load
        // whose offset it feeds costs the wave five wait states (s_nop 4) per row
        int soff[ST_TH];
#if ST_SOFF_HOIST
        st_for([&](auto U) { soff[U] = __builtin_amdgcn_readlane(rows, U); }, std::make_integer_sequence<int, ST_TH>{});
#endif
        st_for([&](auto U) {
            uint32_t cur = ahead[U % LA];
            if constexpr (BP) {
                cur = nxt;
                if (U + 1 < ST_TH) nxt = unpack(ahead[(U + 1) % LA]);
            }
            // the row requested here is consumed only if it lies inside the segment: in the last group
            // the requests of steps U >= ST_TH - LA would read past it (wave-uniform; none for SEGT 1)
            if (U < ST_TH - LA || (SEGT > 1 && i + 1 < ntl)) {
#if ST_SOFF_HOIST
                ahead[U % LA] = load(soff[U]);
#else
                (void)soff;
                ahead[U % LA] = load(__builtin_amdgcn_readlane(rows, U));
#endif
            }
            step(P5{}, k0 + U, cur, U);
        }, std::make_integer_sequence<int, ST_TH>{});
        // the 16 row counts of tile A (lanes 0..15) and B (16..31) are contiguous
        const int tileA = (ys / ST_TH + i) * ntx + 2 * sxi;
        if (lane < (hasB ? 2 * ST_TH : ST_TH) && !(ST_PROBE_NOSTORE & 2)) tilerows[tileA * ST_TH + lane] = (uint8_t)trows;
#if ST_KEYS_LDS
        {
            // the group's keys: tile A's toffA from slot 0, tile B's toffB from ST_TCAP (tile A + 1's
            // region of cand), copied out in order by consecutive lanes.  LDS operations of one wave
            // complete in order, so the next group's writes cannot overtake these reads.
            // ST_HIST_FLUSH (and always in the FLAT form): each flushed key's histogram count here
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            uint64_t* __restrict__ dst = cand + (size_t)tileA * ST_TCAP;
            constexpr bool hf = (FLAT || ST_HIST_FLUSH) && !NH;
            for (int j = lane; j < toffA; j += 64) {
                const uint64_t kv = wkeys[j];
                if (!(ST_PROBE_NOSTORE & 2)) dst[j] = kv;
                if constexpr (hf) st_atomic_add(&hist[min(((uint32_t)(kv >> 32) - thr_bits) >> 15, (uint32_t)(VO_HIST_BINS - 1))], 1u);
            }
            for (int j = lane; j < toffB; j += 64) {
                const uint64_t kv = wkeys[ST_TCAP + j];
                if (!(ST_PROBE_NOSTORE & 2)) dst[ST_TCAP + j] = kv;
                if constexpr (hf) st_atomic_add(&hist[min(((uint32_t)(kv >> 32) - thr_bits) >> 15, (uint32_t)(VO_HIST_BINS - 1))], 1u);
            }
        }
#endif
#if ST_DIAG & 2
        // per tile: the sum over its keys of mix64(key ^ slot << 48), lanes 0..31 tile A, 32..63 tile B
#pragma unroll
        for (int off = 1; off < 32; off <<= 1) dck += __shfl_xor(dck, off);
        if (d.tile_ck && (lane == 0 || (lane == 32 && hasB)))
            d.tile_ck[(size_t)z * d.ntiles + tileA + (lane >> 5)] = dck;
        dck = 0ull;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            sck += __shfl_xor(sck, off);
            rck += __shfl_xor(rck, off);
        }
        if (d.diag_src && lane == 0 && dfr < VO_DIAG_FRAMES) {
            d.diag_src[(size_t)dfr * d.ntiles + tileA] = sck;
            d.diag_resp[(size_t)dfr * d.ntiles + tileA] = rck;
        }
        sck = 0ull; rck = 0ull;
#elif ST_DIAG & 4
        // per lane group of 16 (lanes 0-15, 16-31: tile A's columns; 32-47, 48-63: tile B's) a word
        // of the (f, tileA) entry: the checksums of the four quarter-waves
        {
            uint32_t q = lsck;
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) q = q * 0x9E3779B1u + (uint32_t)__shfl_xor((int)q, off);
            const uint32_t q0 = __shfl(q, 0), q1 = __shfl(q, 16), q2 = __shfl(q, 32), q3 = __shfl(q, 48);
            if (d.diag_src && lane == 0 && dfr < VO_DIAG_FRAMES) {
                d.diag_src[(size_t)dfr * d.ntiles + tileA] = ((unsigned long long)q1 << 32) | q0;
                if (hasB) d.diag_src[(size_t)dfr * d.ntiles + tileA + 1] = ((unsigned long long)q3 << 32) | q2;
            }
        }
        lsck = 0u;
#endif
    }
}

#if ST_NOPK && defined(__HIP_DEVICE_COMPILE__)
#pragma clang attribute pop
#endif

// ---------------------------------------------------------------------------
// select: exact top-N of the candidate keys + raster sort (1 workgroup of 1024)
// Equivalent to popping N times from std::priority_queue<tuple<float,int,int>>
// (corner_detection_parallel_GPU.cpp:147,182-186) then std::sort by (row, col)
// (feature_extraction_parallel_GPU.cpp:259-265).
// ---------------------------------------------------------------------------
#define SEL_MAX 4096
#ifndef SEL_DOT4
#define SEL_DOT4 1
#endif
#define BND_CAP 2048
#define SEL_MAX_TILES 3072
#define SEL_LDS_BITS 65536

template <typename T, bool ASC>
__device__ void bitonic_lds(T* a, int n_pow2)
{
    for (int k = 2; k <= n_pow2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n_pow2; i += blockDim.x) {
                int ixj = i ^ j;
                if (ixj > i) {
                    T x = a[i], y = a[ixj];
                    bool up = ((i & k) == 0) == ASC;
                    if ((x > y) == up) { a[i] = y; a[ixj] = x; }
                }
            }
            __syncthreads();
        }
    }
}

// Dynamic LDS layout of k_select (bytes; host and device derive it from the tile count).
struct SelLayout {
    int rows, tpre, segw, bits, chunk, keys, key_cap, hist, total;
};
__host__ __device__ inline SelLayout sel_layout(int ntiles, int lds_bytes)
{
    auto al = [](int v) { return (v + 15) & ~15; };
    SelLayout L;
    const int nseg = ntiles * ST_TH;
    L.rows = 0;
    L.tpre = L.rows + al(ntiles * 16);
    L.segw = L.tpre + al((ntiles + 1) * 4);
    const int segb = al(nseg > BND_CAP * 8 ? nseg : BND_CAP * 8);     // u8 counts, aliased by boundary keys
    L.bits = L.segw + segb;
    L.chunk = L.bits + SEL_LDS_BITS / 8;                      // u16 prefix per 4 segments
    L.keys = L.chunk + al(((nseg + 3) / 4) * 2);
    // the LDS histogram (lhist launches) at the end, if 1024 keys still fit before it (a small
    // VO_SEL_LDS_KB request: no LDS histogram, the stencil's)
    L.hist = lds_bytes - VO_HIST_BINS * 4;
    if (L.hist - L.keys < 1024 * 8) L.hist = -1;
    L.key_cap = ((L.hist >= 0 ? L.hist : lds_bytes) - L.keys) / 8;
    L.total = lds_bytes;
    return L;
}

__device__ __forceinline__ uint32_t sel_bin(uint64_t key, uint32_t thr_bits)
{
    uint32_t bin = ((uint32_t)(key >> 32) - thr_bits) >> 15;
    return bin > VO_HIST_BINS - 1 ? VO_HIST_BINS - 1 : bin;
}

// select: exact top-N of the NMS survivors by (R,row,col) descending, emitted in raster
// order (feature_extraction_parallel_GPU.cpp:235-265).  One workgroup; every phase is
// parallel over keys (independent loads) -- no per-thread serial walks:
//   A  per-tile row counts -> LDS, tile totals -> block scan (compact key index g, tile order)
//   B  stage the C keys compactly (LDS if they fit, else a global scratch array)
//   C  boundary bin from the stencil histogram; its keys ranked -> exact threshold key Tb
//   D  selected-key bitmap (ballots) + per-(row, tile) selected counts (u8, LDS atomics)
//   E  chunked block scan over the (row, tile) segments in raster order
//   F  each selected key computes its raster position directly and writes its keypoint
// slot of frame f0 + z of an extract batch (vo_internal.h: ring slot, or a stage slot)
__device__ __forceinline__ int ext_slot(const VoDev& d, int f0, int z, int slot_override)
{
    return slot_override >= 0 ? slot_override : (f0 + z) % VO_RING;
}

// lhist: the batch's stencil wrote no histogram (k_stencil NH): it is built here, in LDS, from the keys
// as phase B stages them (one LDS atomic per key), and the global one is neither read nor cleared
__global__ void __launch_bounds__(1024) k_select(VoDev d, int f0, int slot_override, int lhist)
{
    // frame z of the batch: its scratch copy (written by k_stencil's z-slice)
    const int z = blockIdx.x;
    const uint8_t* tilerows = d.tilerows + (size_t)z * d.ntiles * ST_TH;
    const uint64_t* cand = d.cand + (size_t)z * d.cand_cap;
    uint32_t* hist = d.hist + (size_t)z * VO_HIST_BINS;
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ uint32_t s_hs[16];
    __shared__ int s_wsum[16];
    __shared__ int s_nbnd, s_b, s_above;
    __shared__ uint64_t s_tb;
    __shared__ int s_slot;
    __shared__ uint32_t s_dh[256];
    __shared__ int s_dsel, s_rem;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int N = d.N;
    const int ntx = (d.W + ST_TW - 1) / ST_TW, nty = (d.H + ST_TH - 1) / ST_TH, ntiles = ntx * nty;
    const int nseg = ntiles * ST_TH;                    // (row, tile-column) segments, raster order
    const SelLayout L = sel_layout(ntiles, d.sel_lds);
    uint4* s_rows = reinterpret_cast<uint4*>(smem + L.rows);
    int* s_tpre = reinterpret_cast<int*>(smem + L.tpre);
    uint32_t* s_segw = reinterpret_cast<uint32_t*>(smem + L.segw);
    uint64_t* s_bnd = reinterpret_cast<uint64_t*>(smem + L.segw);        // phase C only
    uint64_t* s_bitsl = reinterpret_cast<uint64_t*>(smem + L.bits);
    uint16_t* s_wpre = reinterpret_cast<uint16_t*>(smem + L.chunk);   // selected keys before 4-segment word w
    uint64_t* s_keys = reinterpret_cast<uint64_t*>(smem + L.keys);
    uint32_t* s_lh = reinterpret_cast<uint32_t*>(smem + L.hist);
    const size_t TCAP = ST_TCAP;
#if LDS_POISON
    // diagnostic build: the whole dynamic LDS and the static words filled with a launch-varying
    // pattern first, so a read of LDS this workgroup did not write shows up as a result change
    {
        const uint32_t pz = (uint32_t)wall_clock64() * 0x9E3779B9u ^ (uint32_t)blockIdx.x;
        uint32_t* w = reinterpret_cast<uint32_t*>(smem);
        for (int i = threadIdx.x; i < d.sel_lds / 4; i += 1024) w[i] = pz + (uint32_t)i * 0x85EBCA6Bu;
        if (threadIdx.x < 16) { s_hs[threadIdx.x] = pz; s_wsum[threadIdx.x] = (int)pz; }
        if (threadIdx.x < 256) s_dh[threadIdx.x] = pz;
        if (threadIdx.x == 0) { s_tb = ((uint64_t)pz << 32) | pz; s_dsel = (int)pz; s_rem = (int)pz; }
        __syncthreads();
    }
#endif
    if (tid == 0) {
        s_nbnd = 0; s_b = -1; s_above = 0;
        s_slot = ext_slot(d, f0, z, slot_override);
    }
    VO_STAMP(d, 1900 + (int)blockIdx.x, 0);
    // A
    const int tpt = (ntiles + 1023) / 1024;            // tiles per thread (<= 3)
    int tt[3] = {0, 0, 0};
    int myC = 0;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
        const int t = tid * tpt + u;
        if (u < tpt && t < ntiles) {
            uint4 rc = reinterpret_cast<const uint4*>(tilerows)[t];
            s_rows[t] = rc;
            const uint32_t w4[4] = {rc.x, rc.y, rc.z, rc.w};
            int tot = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                tot += (int)(w4[q] & 0xFF) + (int)((w4[q] >> 8) & 0xFF) + (int)((w4[q] >> 16) & 0xFF) + (int)(w4[q] >> 24);
            tt[u] = tot;
            myC += tot;
        }
    }
    int incl = myC;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int v = __shfl_up(incl, off);
        if (lane >= off) incl += v;
    }
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    int base = incl - myC;
    int C = 0;
    for (int w = 0; w < 16; ++w) { if (w < wave) base += s_wsum[w]; C += s_wsum[w]; }
#pragma unroll
    for (int u = 0; u < 3; ++u) {
        const int t = tid * tpt + u;
        if (u < tpt && t < ntiles) { s_tpre[t] = base; base += tt[u]; }
    }
    if (tid == 0) s_tpre[ntiles] = C;
    const bool bits_lds = C <= SEL_LDS_BITS;
    uint64_t* bits = bits_lds ? s_bitsl : d.selbits + (size_t)z * (d.cand_cap / 64 + 1);
    for (int w = tid; w < (C + 63) / 64; w += 1024) bits[w] = 0ull;
    if (lhist)
        for (int i = tid; i < VO_HIST_BINS; i += 1024) s_lh[i] = 0u;
    __syncthreads();
    // B
    const bool staged = C <= L.key_cap;
    uint64_t* keys = staged ? s_keys : d.ckeys + (size_t)z * d.cand_cap;
    // a thread per tile copies the tile's keys to their compact positions (the keys of a tile
    // are contiguous in both; a binary search of the tile per key cost ten dependent LDS reads).
    // SL_STAGE2: two threads per tile (every other key), eight loads in flight per thread -- a
    // KITTI tile's ~14 keys in one round trip, and all 1024 threads busy (528 tiles)
#if SL_STAGE2 && !ST_DIAG
    for (int t2 = tid; t2 < 2 * ntiles; t2 += 1024) {
        const int t = t2 >> 1, h = t2 & 1;
        const int b = s_tpre[t], n = s_tpre[t + 1] - b;
        const uint64_t* src = cand + (size_t)t * TCAP;
        for (int i = h; i < n; i += 16) {
            uint64_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = i + 2 * u < n ? src[i + 2 * u] : 0ull;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (i + 2 * u < n) {
                    keys[b + i + 2 * u] = v[u];
                    if (lhist) atomicAdd(&s_lh[sel_bin(v[u], d.thr_bits)], 1u);
                }
        }
    }
    if (false)
#endif
    for (int t = tid; t < ntiles; t += 1024) {
        const int b = s_tpre[t], n = s_tpre[t + 1] - b;
        const uint64_t* src = cand + (size_t)t * TCAP;
#if ST_DIAG
        unsigned long long ck = 0ull;
        uint32_t prev_lo = 0u;
        int bad = -1;
        const int tr = t / ntx, tx = t % ntx;
#endif
        for (int i = 0; i < n; i += 4) {
            uint64_t v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = i + u < n ? src[i + u] : 0ull;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u < n) {
                    keys[b + i + u] = v[u];
                    if (lhist) atomicAdd(&s_lh[sel_bin(v[u], d.thr_bits)], 1u);
                }
#if ST_DIAG
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u < n) {
                    // the slot index: tile A's keys from 0, tile B's from ST_TCAP (k_stencil base)
                    const uint64_t slot = (uint64_t)(i + u) + ((tx & 1) ? ST_TCAP : 0);
                    ck += mix64(v[u] ^ (slot << 48));
                    const uint32_t lo = (uint32_t)v[u], row = lo >> 16, col = lo & 0xFFFF;
                    const bool ok = (int)row / ST_TH == tr && (int)col / ST_TW == tx && (uint32_t)(v[u] >> 32) > d.thr_bits &&
                                    (i + u == 0 || lo > prev_lo);
                    if (!ok && bad < 0) bad = i + u;
                    prev_lo = lo;
                }
#endif
        }
#if ST_DIAG
        if (d.diag_tile && f0 + z < VO_DIAG_FRAMES) d.diag_tile[(size_t)(f0 + z) * ntiles + t] = ck;
        if ((ST_DIAG & 2) && d.dbg && d.tile_ck) {
            const unsigned long long want = d.tile_ck[(size_t)z * ntiles + t];
            atomicAdd(&d.dbg[24000], 1ull);
            if (want != ck || bad >= 0) {
                atomicAdd(&d.dbg[want != ck ? 24001 : 24002], 1ull);
                if (atomicCAS(&d.dbg[24003], 0ull, (unsigned long long)(f0 + z + 1)) == 0ull) {
                    d.dbg[24004] = (unsigned long long)t;
                    d.dbg[24005] = want;
                    d.dbg[24006] = ck;
                    d.dbg[24007] = (unsigned long long)n;
                    d.dbg[24008] = (unsigned long long)(bad + 1);
                    for (int i = 0; i < n && i < 24; ++i) d.dbg[24010 + i] = src[i];
                }
            }
        }
#endif
    }
    // tests only (VO_FAULT_INJECT=1): N counts more in the top bin than the tiles hold keys, as
    // k_inject_hist adds to a stencil-built histogram -- the consistency check below must fire
    if (lhist && d.fault_inject && tid == 0) atomicAdd(&s_lh[VO_HIST_BINS - 1], (uint32_t)N);
    __syncthreads();
#if ST_DIAG
    if (d.diag_keys && f0 + z < VO_DIAG_FRAMES)
        for (int g = tid; g < VO_DIAG_KEYS; g += 1024)
            d.diag_keys[(size_t)(f0 + z) * VO_DIAG_KEYS + g] = g < C ? keys[g] : 0ull;
#endif
    VO_STAMP(d, 1900 + (int)blockIdx.x, 1);
    // C (the histogram is read for every frame: its total must equal C, the consistency check)
    int b = -1;
    uint64_t Tb = 0ull;
    uint32_t h[4], hs = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) { h[q] = lhist ? s_lh[4 * tid + q] : hist[4 * tid + q]; hs += h[q]; }
    uint32_t suf = hs;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t v = __shfl_down(suf, off);
        if (lane + off < 64) suf += v;
    }
    if (lane == 0) s_hs[wave] = suf;
    __syncthreads();
    uint32_t htot = 0u;                                 // the histogram's total: the keys the stencil counted
    for (int w = 0; w < 16; ++w) htot += s_hs[w];
    if (C > N) {
        uint32_t above = suf - hs;
        for (int w = wave + 1; w < 16; ++w) above += s_hs[w];
        uint32_t run = above;
        for (int q = 3; q >= 0; --q) {
            if (run < (uint32_t)N && run + h[q] >= (uint32_t)N) { s_b = 4 * tid + q; s_above = (int)run; }
            run += h[q];
        }
        __syncthreads();
        b = s_b;
        VO_STAMP(d, 1900 + (int)blockIdx.x, 2);
        for (int g0 = tid; g0 < C; g0 += 4 * 1024) {
            uint64_t v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = g0 + u * 1024 < C ? keys[g0 + u * 1024] : 0ull;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (g0 + u * 1024 < C && (int)sel_bin(v[u], d.thr_bits) == b) {
                    int p = atomicAdd(&s_nbnd, 1);
                    if (p < BND_CAP) s_bnd[p] = v[u];
                }
            }
        }
        __syncthreads();
        VO_STAMP(d, 1900 + (int)blockIdx.x, 3);
        const int nb = s_nbnd;
        // the need-th largest boundary key: the one with exactly need-1 larger keys
        const int need = N - s_above;
        Tb = ~0ull;
        if (nb > BND_CAP && need > 0) {
            // boundary bin too large to rank in LDS (periodic patterns: many equal responses):
            // radix select over the bin's full 64-bit keys, 8 bits per pass from the top
            uint64_t prefix = 0ull, pmask = 0ull;
            int rem = need;
            for (int shift = 56; shift >= 0; shift -= 8) {
                if (tid < 256) s_dh[tid] = 0u;
                __syncthreads();
                for (int g = tid; g < C; g += 1024) {
                    const uint64_t v = keys[g];
                    if ((int)sel_bin(v, d.thr_bits) == b && (v & pmask) == prefix)
                        atomicAdd(&s_dh[(v >> shift) & 0xFF], 1u);
                }
                __syncthreads();
                if (tid == 0) {
                    int run = 0, dsel = 0;
                    for (int dd = 255; dd >= 0; --dd) {
                        const int h = (int)s_dh[dd];
                        if (run + h >= rem) { dsel = dd; break; }
                        run += h;
                    }
                    s_dsel = dsel;
                    s_rem = rem - run;
                }
                __syncthreads();
                prefix |= (uint64_t)s_dsel << shift;
                pmask |= 0xFFull << shift;
                rem = s_rem;
                __syncthreads();
            }
            Tb = prefix;                               // keys are unique: one key matches all 64 bits
        } else if (need > 0) {
            for (int e = tid; e < nb; e += 1024) {
                const uint64_t ke = s_bnd[e];
                int rank = 0;
                for (int f = 0; f < nb; ++f) rank += s_bnd[f] > ke;
                if (rank == need - 1) s_tb = ke;        // keys are unique (they carry row, col)
            }
            __syncthreads();
            Tb = s_tb;
        }
        if (tid == 0 && d.dbg) d.dbg[1990 * 16 + 10] = (unsigned long long)nb;
    }
    __syncthreads();                                    // s_bnd aliases the segment counts
    for (int w = tid; w < (nseg + 3) / 4; w += 1024) s_segw[w] = 0u;
    __syncthreads();
    VO_STAMP(d, 1900 + (int)blockIdx.x, 4);
    auto selected = [&](uint64_t key) -> bool {
        if (b < 0) return true;
        const int bin = (int)sel_bin(key, d.thr_bits);
        return bin > b || (bin == b && key >= Tb);
    };
    // D
    const int nround = (C + 1023) / 1024;
    for (int r0 = 0; r0 < nround; r0 += 4) {
        uint64_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int g = (r0 + u) * 1024 + tid;
            v[u] = g < C ? keys[g] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (r0 + u >= nround) break;
            const int g = (r0 + u) * 1024 + tid;
            const bool sel = g < C && selected(v[u]);
            const uint64_t bal = __ballot(sel);
            if (lane == 0 && ((r0 + u) * 1024 + wave * 64) < C) bits[((r0 + u) * 1024 + wave * 64) >> 6] = bal;
            if (sel) {
                const int row = (int)((v[u] >> 16) & 0xFFFF), col = (int)(v[u] & 0xFFFF);
                const int seg = row * ntx + col / ST_TW;
                atomicAdd(&s_segw[seg >> 2], 1u << (8 * (seg & 3)));
            }
        }
    }
    __syncthreads();
    // E: exclusive prefix of the selected counts per 4-segment word; thread tid owns words
    //    [tid*cw, tid*cw+cw) (segment counts are u8, four to a word)
    auto wordsum = [](uint32_t w) -> int {
        const uint32_t p = (w & 0x00FF00FFu) + ((w >> 8) & 0x00FF00FFu);
        return (int)((p & 0xFFFF) + (p >> 16));
    };
    {
        const int nw = (nseg + 3) / 4, cw = (nw + 1023) / 1024;
        const int w0 = min(tid * cw, nw), w1 = min(w0 + cw, nw);
        int mine = 0;
        for (int w = w0; w < w1; ++w) mine += wordsum(s_segw[w]);
        int inc2 = mine;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            int v = __shfl_up(inc2, off);
            if (lane >= off) inc2 += v;
        }
        if (lane == 63) s_wsum[wave] = inc2;
        __syncthreads();
        int pre = inc2 - mine;
        for (int w = 0; w < wave; ++w) pre += s_wsum[w];
        for (int w = w0; w < w1; ++w) {
            s_wpre[w] = (uint16_t)pre;                  // <= N <= 4096 selected keys
            pre += wordsum(s_segw[w]);
        }
    }
    __syncthreads();
    VO_STAMP(d, 1900 + (int)blockIdx.x, 5);
    // F
    const int slot = s_slot;
    int2* out = d.kps + (size_t)slot * N;
    for (int r0 = 0; r0 < nround; r0 += 4) {
        uint64_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int g = (r0 + u) * 1024 + tid;
            v[u] = g < C ? keys[g] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int g = (r0 + u) * 1024 + tid;
            if (g >= C || !((bits[g >> 6] >> (g & 63)) & 1ull)) continue;
            const int row = (int)((v[u] >> 16) & 0xFFFF), col = (int)(v[u] & 0xFFFF);
            const int x = col / ST_TW, r = row & (ST_TH - 1), t = (row / ST_TH) * ntx + x;
            const int seg = row * ntx + x;
            // first compact index of this (row, tile) segment
            const uint4 rc = s_rows[t];
            const uint32_t w4[4] = {rc.x, rc.y, rc.z, rc.w};
            int start = 0;
#if SEL_DOT4
            // the row counts below r (bytes of the four words): each word masked to its bytes below
            // r (a 64-bit shift covers the whole-word and empty cases) and summed by v_dot4_u32_u8
            // -- no compare / select per row
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int sh = 8 * min(max(r - 4 * k, 0), 4);
                const uint32_t m = (uint32_t)(0xFFFFFFFFull >> (32 - sh));
                start = (int)__builtin_amdgcn_udot4(w4[k] & m, 0x01010101u, (uint32_t)start, false);
            }
#else
#pragma unroll
            for (int q = 0; q < ST_TH; ++q)
                if (q < r) start += (int)((w4[q >> 2] >> (8 * (q & 3))) & 0xFF);
#endif
            const int gs = s_tpre[t] + start;
            // selected keys before g inside the segment
            int within = 0;
            for (int wi = gs >> 6; wi <= (g >> 6); ++wi) {
                uint64_t m = bits[wi];
                if (wi == (gs >> 6)) m &= ~0ull << (gs & 63);
                if (wi == (g >> 6)) m &= (g & 63) ? (~0ull >> (64 - (g & 63))) : 0ull;
                within += __popcll(m);
            }
            // the segment's start: its word's prefix plus the counts of the word's lower segments
            const uint32_t sw = s_segw[seg >> 2] & ((1u << (8 * (seg & 3))) - 1u);
            const int pos = (int)s_wpre[seg >> 2] + wordsum(sw) + within;
            if (pos < N) out[pos] = make_int2(col, row);  // < N by construction (corrupt input: no stray store)
        }
    }
    VO_STAMP(d, 1900 + (int)blockIdx.x, 6);
    // select is the histogram's only reader: leave it zeroed for the next frame's stencil
    if (!lhist)
        for (int i = tid; i < VO_HIST_BINS; i += 1024) hist[i] = 0u;
    if (tid == 0) {
        // consistency: the histogram counts exactly the keys the tiles hold (round 4's r4j stencil
        // counted margin-row maxima it never stored, tests/test_select_consistency.py), and the
        // keypoints emitted are min(C, N).  A failure is a library defect, never a capacity limit:
        // the frame gets 0 keypoints (no later kernel reads a slot entry nobody wrote), its own
        // status, and the context's error counter, which the host turns into VO_ERR_INTERNAL
        int sel = 0;
        for (int w = 0; w < 16; ++w) sel += s_wsum[w];
        const bool bad = htot != (uint32_t)C || sel != (C < N ? C : N);
        d.ext_n[slot] = bad ? 0 : (C < N ? C : N);
        d.ext_st[slot] = bad ? VO_STATUS_INCONSISTENT : VO_STATUS_OK;
        if (bad) atomicAdd(d.ctr + VO_CTR_ERR, 1u);
    }
}

// ---------------------------------------------------------------------------
// in-launch hand-off: the last workgroup to arrive consumes what the others produced.
// Valid form of MI355X_MICROARCH.md "Workgroup dispatch ... visibility" (table row 1):
// payload stored sc1 (agent-scope relaxed atomic stores), every storing wave drains
// vmcnt(0), one lane per workgroup adds to ONE unsharded counter, the workgroup whose
// add returns total-1 loads the payload with sc1 loads only.  The counter is reset by
// that last workgroup for the next launch (kernel boundary orders it).
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(1))) int gi32;
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ void st_sc1(int* p, int v)
{
    __hip_atomic_store((gi32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_sc1(const int* p)
{
    return __hip_atomic_load((gi32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool arrive_last(unsigned* ctr, unsigned total, unsigned* s_flag)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned prev = __hip_atomic_fetch_add((gu32*)ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *s_flag = (prev == total - 1) ? 1u : 0u;
    }
    __syncthreads();
    return *s_flag != 0u;
}

// Cross-queue hand-off to the other HIP queue's stream-wait-value packet (vo_api.cpp
// enqueue_frame): every wave drains its stores, the workgroup meets, then one lane stores the
// frame counter with a system-scope release (L2 write-back, then a write-through store the
// command processor reads from memory).  Workgroups other than the caller must already have
// published their stores at agent scope (release fence before arrive_last).
__device__ __forceinline__ void publish_seq(unsigned* flag, unsigned v)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store((gu32*)flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// Banded select: the exact top-N of a frame's NMS survivors by (R, row, col) descending, emitted in
// raster order (corner_detection_parallel_GPU.cpp:146-188, feature_extraction_parallel_GPU.cpp:
// 235-265), on VO_SEL_BANDS workgroups per frame instead of one.  Workgroup w owns band w: a
// contiguous run of tile rows, so the band's keys precede band w + 1's in raster order.
//   k_select_count  every workgroup finds the boundary bin b of the stencil's histogram (the bin
//                   where the count from the top reaches N), counts its band's keys above b and
//                   appends the band's keys of bin b to the frame's boundary list; the last to
//                   arrive ranks the boundary list (the (N - above)-th largest key is the
//                   threshold Tb; keys carry row and col, so they are unique), and turns the band
//                   counts into each band's first output position.
//   k_select_emit   each band counts its selected keys per (row, tile) segment, scans the
//                   segments in raster order and writes every selected key at its position.
// A tile's keys are read by one wave, lane = key (tile-local raster order: ascending row, then
// column), so a segment's keys are contiguous lanes and a key's rank inside its segment is a
// popcount of the wave's selection ballot.
// ---------------------------------------------------------------------------
#define SL_T 256
#define SL_RANK_MAX 256        // boundary lists up to this size are ranked pairwise in LDS; longer
                               // ones by a radix select (8 bits a pass, from the top)
#define SL_TOF_CAP 8192        // band keys up to this many: a key's tile from an LDS table (else a binary search)
typedef __attribute__((address_space(1))) unsigned long long gu64;
__device__ __forceinline__ void st_sc1_u64(uint64_t* p, uint64_t v)
{
    __hip_atomic_store((gu64*)p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1_u64(const uint64_t* p)
{
    return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// band w of the frame: tile rows [ty0, ty1)
__host__ __device__ inline void sel_band(int nty, int w, int& ty0, int& ty1)
{
    const int nbr = (nty + VO_SEL_BANDS - 1) / VO_SEL_BANDS;
    ty0 = w * nbr < nty ? w * nbr : nty;
    ty1 = ty0 + nbr < nty ? ty0 + nbr : nty;
}
// dynamic LDS of the banded select kernels (bytes), for bands of at most ntm tiles (nbr tile rows)
struct SelBandLayout {
    int rows, pre, tof, bits, seg, total;
};
__host__ __device__ inline SelBandLayout sel_band_layout(int ntx, int nty)
{
    auto al = [](int v) { return (v + 15) & ~15; };
    const int nbr = (nty + VO_SEL_BANDS - 1) / VO_SEL_BANDS, ntm = nbr * ntx;
    SelBandLayout L;
    L.rows = 0;                                              // uint4 row counts per band tile
    L.pre = al(16 * ntm);                                    // int: first compact key index per tile (+ total)
    L.tof = L.pre + al(4 * (ntm + 1));                       // u16: tile of each compact key
    L.bits = L.tof + al(2 * SL_TOF_CAP);                     // u64: selected-key bitmap
    L.seg = L.bits + al(8 * (ntm * ST_TCAP / 64 + 2));       // u16: per (row, tile) segment, pairs per word
    L.total = L.seg + al(2 * (nbr * ST_TH * ntx + 1));
    return L;
}
// the fused select's LDS past the band layout: the band's keys (u64, SL_TOF_CAP) and its boundary-bin
// keys' compact indices (int, SL_TOF_CAP)
__host__ __device__ inline int sel_fused_kbuf(int ntx, int nty) { return (sel_band_layout(ntx, nty).total + 15) & ~15; }
__host__ __device__ inline int sel_fused_lds(int ntx, int nty) { return sel_fused_kbuf(ntx, nty) + 12 * SL_TOF_CAP; }
__device__ __forceinline__ int row_bytes(uint4 rc)
{
    uint32_t s = 0u;
    s = __builtin_amdgcn_udot4(rc.x, 0x01010101u, s, false);
    s = __builtin_amdgcn_udot4(rc.y, 0x01010101u, s, false);
    s = __builtin_amdgcn_udot4(rc.z, 0x01010101u, s, false);
    s = __builtin_amdgcn_udot4(rc.w, 0x01010101u, s, false);
    return (int)s;
}
// block-wide inclusive suffix sum over SL_T threads (s_w: 4 words)
__device__ __forceinline__ uint32_t sel_suffix(uint32_t v, uint32_t* s_w)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t suf = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t u = __shfl_down(suf, off);
        if (lane + off < 64) suf += u;
    }
    if (lane == 0) s_w[wave] = suf;
    __syncthreads();
    for (int w = wave + 1; w < SL_T / 64; ++w) suf += s_w[w];
    __syncthreads();
    return suf;
}
// the band's tile table: row counts, each tile's first compact key index (keys numbered in tile
// order), and each key's tile when the band holds at most SL_TOF_CAP keys.  Thread tid owns band
// tiles [tid tpt, tid tpt + tpt).  Returns the band's key count.
__device__ int sel_band_table(const uint8_t* tilerows, int t0, int nt, uint4* s_rows, int* s_pre, uint16_t* s_tof,
                              uint32_t* s_w)
{
    const int tid = threadIdx.x, tpt = (nt + SL_T - 1) / SL_T;
    const int k0 = min(tid * tpt, nt), k1 = min(k0 + tpt, nt);
    int mine = 0;
    for (int k = k0; k < k1; ++k) {
        const uint4 rc = *reinterpret_cast<const uint4*>(tilerows + (size_t)(t0 + k) * ST_TH);
        s_rows[k] = rc;
        const int c = row_bytes(rc);
        s_pre[k] = c;
        mine += c;
    }
    const uint32_t after = sel_suffix((uint32_t)mine, s_w);
    __shared__ int s_total;
    if (tid == 0) s_total = (int)after;
    __syncthreads();
    const int total = s_total;
    int base = total - (int)after;
    for (int k = k0; k < k1; ++k) {
        const int c = s_pre[k];
        s_pre[k] = base;
        if (total <= SL_TOF_CAP)
            for (int i = 0; i < c; ++i) s_tof[base + i] = (uint16_t)k;
        base += c;
    }
    if (tid == 0) s_pre[nt] = total;
    __syncthreads();
    return total;
}
// band tile of compact key g
__device__ __forceinline__ int sel_tile_of(int g, int total, int nt, const int* s_pre, const uint16_t* s_tof)
{
    if (total <= SL_TOF_CAP) return s_tof[g];
    int lo = 0, hi = nt - 1;                         // the last tile whose first key is <= g
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_pre[mid] <= g) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// fused (the per-frame call's k_select_fused): the last band to arrive also publishes ctl->ready
// after writing the threshold and the band positions, for the other bands waiting in the same launch
// kbuf (the fused select, a band of at most SL_TOF_CAP keys): the band's keys are kept in LDS as they
// are read (kbuf[g], compact index g), for the emit in the same launch.  Returns whether this band
// arrived last (ranked the boundary keys and published); *total_out / *b_out: the band's key count
// and the boundary bin
__device__ __forceinline__ bool sel_count_body(const VoDev& d, int f0, int slot_override, int z, int w,
                                               unsigned char* smem, bool fused, uint64_t* kbuf = nullptr,
                                               int* total_out = nullptr, int* b_out = nullptr)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int N = d.N;
    const int ntx = (d.W + ST_TW - 1) / ST_TW, nty = (d.H + ST_TH - 1) / ST_TH;
    const SelBandLayout L = sel_band_layout(ntx, nty);
    uint4* s_rows = reinterpret_cast<uint4*>(smem + L.rows);
    int* s_pre = reinterpret_cast<int*>(smem + L.pre);
    uint16_t* s_tof = reinterpret_cast<uint16_t*>(smem + L.tof);
    const uint8_t* tilerows = d.tilerows + (size_t)z * d.ntiles * ST_TH;
    const uint64_t* cand = d.cand + (size_t)z * d.cand_cap;
    uint32_t* hist = d.hist + (size_t)z * VO_HIST_BINS;
    VoSelCtl* ctl = d.selctl + z;
    uint64_t* bnd = d.ckeys + (size_t)z * d.cand_cap;            // the frame's boundary-bin keys
    __shared__ uint32_t s_w[4];
    __shared__ int s_b, s_above, s_C, s_rem, s_dsel;
    __shared__ uint32_t s_last;
    __shared__ uint64_t s_tb;
    __shared__ uint64_t s_key[SL_RANK_MAX];
    __shared__ uint32_t s_dh[256];
    __shared__ int s_cnt[VO_SEL_BANDS];
    int ty0, ty1;
    sel_band(nty, w, ty0, ty1);
    const int t0 = ty0 * ntx, nt = (ty1 - ty0) * ntx;
    VO_STAMP(d, 1960 + w, 0);                            // (stamps: the per-frame select's band w)
    // 1. boundary bin: thread tid holds bins 16 tid .. 16 tid + 15 (loads issued with the band table's)
    uint32_t h[16], hs = 0u;
    {
        const uint4* hp = reinterpret_cast<const uint4*>(hist) + 4 * tid;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 v = hp[q];
            h[4 * q] = v.x; h[4 * q + 1] = v.y; h[4 * q + 2] = v.z; h[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) hs += h[q];
    }
    const int total = sel_band_table(tilerows, t0, nt, s_rows, s_pre, s_tof, s_w);
    VO_STAMP(d, 1960 + w, 1);
    if (tid == 0) { s_b = -1; s_above = 0; }
    const uint32_t suf = sel_suffix(hs, s_w);            // keys in bins >= 16 tid
    if (tid == 0) s_C = (int)suf;
    __syncthreads();
    const int C = s_C;
    if (C > N) {
        uint32_t run = suf - hs;                         // keys in bins above this thread's
#pragma unroll
        for (int q = 15; q >= 0; --q) {
            if (run < (uint32_t)N && run + h[q] >= (uint32_t)N) { s_b = 16 * tid + q; s_above = (int)run; }
            run += h[q];
        }
    }
    __syncthreads();
    const int b = s_b;
    if (total_out) { *total_out = total; *b_out = b; }
    if (total > SL_TOF_CAP) kbuf = nullptr;
    VO_STAMP(d, 1960 + w, 2);
    // 2. the band's keys above bin b, and its keys of bin b appended to the frame's boundary list
    int D = 0;
    if (b < 0) {
        D = tid == 0 ? total : 0;
    } else {
        for (int g0 = 0; g0 < total; g0 += 4 * SL_T) {
            uint64_t key[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int g = g0 + u * SL_T + tid;
                key[u] = 0ull;
                if (g < total) {
                    const int k = sel_tile_of(g, total, nt, s_pre, s_tof);
                    key[u] = cand[(size_t)(t0 + k) * ST_TCAP + (g - s_pre[k])];
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int g = g0 + u * SL_T + tid;
                if (kbuf && g < total) kbuf[g] = key[u];
                const int bin = g < total ? (int)sel_bin(key[u], d.thr_bits) : -1;
                D += bin > b ? 1 : 0;
                const unsigned long long m = ballot64(bin == b);
                if (m) {
                    uint32_t p0 = 0u;
                    if (lane == 0) p0 = atomicAdd(&ctl->nbnd, (unsigned)__popcll(m));
                    p0 = __shfl(p0, 0);
                    if (bin == b)
                        st_sc1_u64(bnd + p0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)), key[u]);
                }
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) D += __shfl_xor(D, off);
    if (lane == 0) s_w[wave] = (uint32_t)D;
    __syncthreads();
    if (tid == 0) {
        st_sc1(&ctl->dcount[w], (int)(s_w[0] + s_w[1] + s_w[2] + s_w[3]));
        st_sc1(&ctl->ktot[w], total);                    // the band's keys by the tile row counts
    }
    VO_STAMP(d, 1960 + w, 3);
    if (!arrive_last(&ctl->arrive, VO_SEL_BANDS, &s_last)) return false;
    // 3. last workgroup of the frame: the threshold key, each band's first position
    const int nbk = (int)__hip_atomic_load((gu32*)&ctl->nbnd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int need = N - s_above;                        // boundary keys to select (b >= 0)
    uint64_t Tb = 0ull;
    const bool in_lds = nbk <= SL_RANK_MAX;
    if (b >= 0) {
        if (in_lds) {
            for (int e = tid; e < nbk; e += SL_T) s_key[e] = ld_sc1_u64(bnd + e);
            __syncthreads();
            for (int e = tid; e < nbk; e += SL_T) {
                const uint64_t ke = s_key[e];
                int rank = 0;
                for (int f = 0; f < nbk; ++f) rank += s_key[f] > ke ? 1 : 0;
                if (rank == need - 1) s_tb = ke;
            }
            __syncthreads();
            Tb = s_tb;
        } else {
            uint64_t prefix = 0ull, pmask = 0ull;
            int rem = need;
            for (int shift = 56; shift >= 0; shift -= 8) {
                s_dh[tid] = 0u;
                __syncthreads();
                for (int e = tid; e < nbk; e += SL_T) {
                    const uint64_t v = ld_sc1_u64(bnd + e);
                    if ((v & pmask) == prefix) atomicAdd(&s_dh[(v >> shift) & 0xFF], 1u);
                }
                __syncthreads();
                // digit tid: keys of the prefix with digit >= tid; the selected digit is the one where
                // that count first reaches rem
                const uint32_t c = s_dh[tid];
                const uint32_t ge = sel_suffix(c, s_w);
                if (ge >= (uint32_t)rem && ge - c < (uint32_t)rem) { s_dsel = tid; s_rem = rem - (int)(ge - c); }
                __syncthreads();
                prefix |= (uint64_t)s_dsel << shift;
                pmask |= 0xFFull << shift;
                rem = s_rem;
                __syncthreads();
            }
            Tb = prefix;                                 // one key matches all 64 bits
        }
    }
    __shared__ int s_ktot[VO_SEL_BANDS];
    if (tid < VO_SEL_BANDS) {
        s_cnt[tid] = ld_sc1(&ctl->dcount[tid]);
        s_ktot[tid] = ld_sc1(&ctl->ktot[tid]);
    }
    __syncthreads();
    if (b >= 0) {
        const int nbr = (nty + VO_SEL_BANDS - 1) / VO_SEL_BANDS;
        for (int e = tid; e < nbk; e += SL_T) {
            const uint64_t v = in_lds ? s_key[e] : ld_sc1_u64(bnd + e);
            if (v >= Tb) atomicAdd(&s_cnt[(int)((v >> 16) & 0xFFFF) / ST_TH / nbr], 1);
        }
    }
    __syncthreads();
    if (tid == 0) {
        int pre = 0;
        for (int k = 0; k < VO_SEL_BANDS; ++k) { ctl->base[k] = pre; pre += s_cnt[k]; }
        ctl->b = b;
        ctl->Tb = Tb;
        ctl->arrive = 0u;                                // for the next launch (the kernel boundary orders it)
        ctl->nbnd = 0u;
        const int slot = ext_slot(d, f0, z, slot_override);
        // consistency (as k_select): the keys the tiles hold (the bands' totals) equal the histogram's
        // total C, and the keypoints the bands will emit (pre) are min(C, N).  A failure gives the
        // frame 0 keypoints (nothing reads a slot entry nobody wrote), VO_STATUS_INCONSISTENT and a
        // count in the context's error counter (VO_ERR_INTERNAL on the host)
        int kt = 0;
        for (int k = 0; k < VO_SEL_BANDS; ++k) kt += s_ktot[k];
        const bool bad = kt != C || pre != (C < N ? C : N);
        d.ext_n[slot] = bad ? 0 : (C < N ? C : N);
        d.ext_st[slot] = bad ? VO_STATUS_INCONSISTENT : VO_STATUS_OK;
        if (bad) atomicAdd(d.ctr + VO_CTR_ERR, 1u);
        if (fused) __hip_atomic_store((gu32*)&ctl->ready, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    VO_STAMP(d, 1968, 0);                                // the last band: ranked and published
    // every band has read the histogram: leave it zeroed for the next frame's stencil
    uint4* hp = reinterpret_cast<uint4*>(hist) + 4 * tid;
#pragma unroll
    for (int q = 0; q < 4; ++q) hp[q] = make_uint4(0u, 0u, 0u, 0u);
    return true;
}

__global__ void __launch_bounds__(SL_T) k_select_count(VoDev d, int f0, int slot_override, int nb)
{
    int z, w;
    if (!xcd_frame(d, VO_SEL_BANDS, nb, z, w)) return;
    extern __shared__ __align__(16) unsigned char smem[];
    sel_count_body(d, f0, slot_override, z, w, smem, false);
}

__device__ __forceinline__ void sel_emit_body(const VoDev& d, int f0, int slot_override, int z, int w,
                                              unsigned char* smem)
{
    __shared__ uint32_t s_w[4];
    const int tid = threadIdx.x, lane = tid & 63;
    const int N = d.N;
    const int ntx = (d.W + ST_TW - 1) / ST_TW, nty = (d.H + ST_TH - 1) / ST_TH;
    const SelBandLayout L = sel_band_layout(ntx, nty);
    uint4* s_rows = reinterpret_cast<uint4*>(smem + L.rows);
    int* s_pre = reinterpret_cast<int*>(smem + L.pre);
    uint16_t* s_tof = reinterpret_cast<uint16_t*>(smem + L.tof);
    uint64_t* s_bits = reinterpret_cast<uint64_t*>(smem + L.bits);
    uint16_t* s_seg = reinterpret_cast<uint16_t*>(smem + L.seg);  // per (row - r0) * ntx + tile column
    uint32_t* s_seg32 = reinterpret_cast<uint32_t*>(smem + L.seg);
    const uint8_t* tilerows = d.tilerows + (size_t)z * d.ntiles * ST_TH;
    const uint64_t* cand = d.cand + (size_t)z * d.cand_cap;
    const VoSelCtl* ctl = d.selctl + z;
    const int b = ctl->b, base = ctl->base[w];
    const uint64_t Tb = ctl->Tb;
    int ty0, ty1;
    sel_band(nty, w, ty0, ty1);
    const int t0 = ty0 * ntx, nt = (ty1 - ty0) * ntx, r0 = ty0 * ST_TH, nseg = (ty1 - ty0) * ST_TH * ntx;
    if (nt <= 0) return;
    VO_STAMP(d, 1960 + w, 5);
    for (int s = tid; s < (nseg + 1) / 2; s += SL_T) s_seg32[s] = 0u;
    const int total = sel_band_table(tilerows, t0, nt, s_rows, s_pre, s_tof, s_w);
    VO_STAMP(d, 1960 + w, 6);
    auto selected = [&](uint64_t key) -> bool {
        if (b < 0) return true;
        const int bin = (int)sel_bin(key, d.thr_bits);
        return bin > b || (bin == b && key >= Tb);
    };
    auto seg_of = [&](uint64_t key, int k) { return ((int)((key >> 16) & 0xFFFF) - r0) * ntx + (t0 + k) % ntx; };
    // 1. selection bitmap (a wave's 64 keys are one word) and selected keys per segment (u16 pairs)
    for (int g0 = 0; g0 < total; g0 += 4 * SL_T) {
        uint64_t key[4];
        int kk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int g = g0 + u * SL_T + tid;
            key[u] = 0ull;
            kk[u] = 0;
            if (g < total) {
                kk[u] = sel_tile_of(g, total, nt, s_pre, s_tof);
                key[u] = cand[(size_t)(t0 + kk[u]) * ST_TCAP + (g - s_pre[kk[u]])];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int g = g0 + u * SL_T + tid;
            if (g0 + u * SL_T >= total) break;
            const bool sel = g < total && selected(key[u]);
            const unsigned long long m = ballot64(sel);
            if (lane == 0 && g < total) s_bits[g >> 6] = m;
            if (sel) {
                const int sg = seg_of(key[u], kk[u]);
                atomicAdd(&s_seg32[sg >> 1], 1u << (16 * (sg & 1)));
            }
        }
    }
    __syncthreads();
    VO_STAMP(d, 1960 + w, 7);
    // 2. exclusive scan of the segments in raster order: thread tid owns [tid cw, tid cw + cw)
    {
        const int cw = (nseg + SL_T - 1) / SL_T;
        const int s0 = min(tid * cw, nseg), s1 = min(s0 + cw, nseg);
        uint32_t mine = 0u;
        for (int s = s0; s < s1; ++s) mine += s_seg[s];
        const uint32_t after = sel_suffix(mine, s_w);    // this thread's and every later thread's
        __shared__ uint32_t s_sum;
        if (tid == 0) s_sum = after;
        __syncthreads();
        uint32_t pre = s_sum - after;
        for (int s = s0; s < s1; ++s) {
            const uint32_t v = s_seg[s];
            s_seg[s] = (uint16_t)pre;                    // <= N <= 4096
            pre += v;
        }
    }
    __syncthreads();
    VO_STAMP(d, 1960 + w, 8);
    // 3. each selected key at base + its segment's start + the selected keys before it in the
    //    segment (contiguous compact indices: a segment is one row of one tile)
    const int slot = ext_slot(d, f0, z, slot_override);
    int2* out = d.kps + (size_t)slot * N;
    for (int g0 = 0; g0 < total; g0 += 4 * SL_T) {
        uint64_t key[4];
        int kk[4];
        bool sel[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int g = g0 + u * SL_T + tid;
            sel[u] = g < total && ((s_bits[g >> 6] >> (g & 63)) & 1ull);
            key[u] = 0ull;
            kk[u] = 0;
            if (sel[u]) {
                kk[u] = sel_tile_of(g, total, nt, s_pre, s_tof);
                key[u] = cand[(size_t)(t0 + kk[u]) * ST_TCAP + (g - s_pre[kk[u]])];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (!sel[u]) continue;
            const int g = g0 + u * SL_T + tid;
            const int row = (int)((key[u] >> 16) & 0xFFFF), col = (int)(key[u] & 0xFFFF);
            const int r = row & (ST_TH - 1);
            // the segment's first compact index: the tile's first plus its row counts below r
            const uint4 rc = s_rows[kk[u]];
            const uint32_t w4[4] = {rc.x, rc.y, rc.z, rc.w};
            int start = s_pre[kk[u]];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int sh = 8 * min(max(r - 4 * q, 0), 4);
                const uint32_t msk = (uint32_t)(0xFFFFFFFFull >> (32 - sh));
                start = (int)__builtin_amdgcn_udot4(w4[q] & msk, 0x01010101u, (uint32_t)start, false);
            }
            // selected keys in [start, g): at most two bitmap words (a segment holds <= 28 keys)
            int within = 0;
            for (int wi = start >> 6; wi <= (g >> 6); ++wi) {
                uint64_t m = s_bits[wi];
                if (wi == (start >> 6)) m &= ~0ull << (start & 63);
                if (wi == (g >> 6)) m &= (g & 63) ? (~0ull >> (64 - (g & 63))) : 0ull;
                within += __popcll(m);
            }
            const int pos = base + (int)s_seg[seg_of(key[u], kk[u])] + within;
            if (pos < N) out[pos] = make_int2(col, row);  // < N by construction
        }
    }
    VO_STAMP(d, 1960 + w, 9);
}

// The fused select's emit for a band of at most SL_TOF_CAP keys (sel_count_body staged them in kbuf and
// left the band table in LDS): the selection bitmap and segment counts of every key outside the
// boundary bin b are known before the threshold key Tb is, so they are built while the last band
// ranks; after the wait only the band's boundary-bin keys (their compact indices in s_bl) are added
// against Tb.  Then the segment scan and the emission as sel_emit_body, keys from LDS.
// wait(): blocks until ctl->ready (false: timed out)
template <typename Wait>
__device__ __forceinline__ void sel_emit_fused(const VoDev& d, int f0, int slot_override, int z, int w,
                                               unsigned char* smem, int total, int b, Wait&& wait)
{
    __shared__ uint32_t s_w[4];
    __shared__ int s_nbl;
    const int tid = threadIdx.x, lane = tid & 63;
    const int N = d.N;
    const int ntx = (d.W + ST_TW - 1) / ST_TW, nty = (d.H + ST_TH - 1) / ST_TH;
    const SelBandLayout L = sel_band_layout(ntx, nty);
    uint4* s_rows = reinterpret_cast<uint4*>(smem + L.rows);
    int* s_pre = reinterpret_cast<int*>(smem + L.pre);
    uint16_t* s_tof = reinterpret_cast<uint16_t*>(smem + L.tof);
    uint64_t* s_bits = reinterpret_cast<uint64_t*>(smem + L.bits);
    uint16_t* s_seg = reinterpret_cast<uint16_t*>(smem + L.seg);
    uint32_t* s_seg32 = reinterpret_cast<uint32_t*>(smem + L.seg);
    const uint64_t* kbuf = reinterpret_cast<const uint64_t*>(smem + sel_fused_kbuf(ntx, nty));
    int* s_bl = reinterpret_cast<int*>(smem + sel_fused_kbuf(ntx, nty) + 8 * SL_TOF_CAP);
    const uint64_t* cand = d.cand + (size_t)z * d.cand_cap;
    const VoSelCtl* ctl = d.selctl + z;
    int ty0, ty1;
    sel_band(nty, w, ty0, ty1);
    const int t0 = ty0 * ntx, nt = (ty1 - ty0) * ntx, r0 = ty0 * ST_TH, nseg = (ty1 - ty0) * ST_TH * ntx;
    // (b < 0: sel_count_body read no key; every key is selected, from the tiles)
    auto key_of = [&](int g, int k) { return b >= 0 ? kbuf[g] : cand[(size_t)(t0 + k) * ST_TCAP + (g - s_pre[k])]; };
    auto seg_of = [&](uint64_t key, int k) { return ((int)((key >> 16) & 0xFFFF) - r0) * ntx + (t0 + k) % ntx; };
    VO_STAMP(d, 1960 + w, 5);
    if (nt > 0) {
        for (int s = tid; s < (nseg + 1) / 2; s += SL_T) s_seg32[s] = 0u;
        if (tid == 0) s_nbl = 0;
        __syncthreads();
        VO_STAMP(d, 1960 + w, 6);
        // 1. bitmap and segment counts of the keys above bin b; bin b's keys listed
        for (int g0 = 0; g0 < total; g0 += SL_T) {
            const int g = g0 + tid;
            bool sel = false;
            if (g < total) {
                const int k = s_tof[g];
                const uint64_t key = key_of(g, k);
                const int bin = b >= 0 ? (int)sel_bin(key, d.thr_bits) : 0;
                sel = b < 0 || bin > b;
                if (sel) {
                    const int sg = seg_of(key, k);
                    atomicAdd(&s_seg32[sg >> 1], 1u << (16 * (sg & 1)));
                } else if (bin == b) {
                    s_bl[atomicAdd(&s_nbl, 1)] = g;
                }
            }
            const unsigned long long m = ballot64(sel);
            if (lane == 0 && g < total) s_bits[g >> 6] = m;
        }
    }
    // 2. the threshold key and the band's first position
    if (!wait()) return;
    const int base = ctl->base[w];
    const uint64_t Tb = ctl->Tb;
    if (nt <= 0) return;
    VO_STAMP(d, 1960 + w, 7);
    // 3. bin b's keys at or above Tb
    for (int i = tid; i < s_nbl; i += SL_T) {
        const int g = s_bl[i];
        const uint64_t key = kbuf[g];
        if (key >= Tb) {
            atomicOr(&s_bits[g >> 6], 1ull << (g & 63));
            const int sg = seg_of(key, s_tof[g]);
            atomicAdd(&s_seg32[sg >> 1], 1u << (16 * (sg & 1)));
        }
    }
    __syncthreads();
    // 4. exclusive scan of the segments in raster order: thread tid owns [tid cw, tid cw + cw)
    {
        const int cw = (nseg + SL_T - 1) / SL_T;
        const int s0 = min(tid * cw, nseg), s1 = min(s0 + cw, nseg);
        uint32_t mine = 0u;
        for (int s = s0; s < s1; ++s) mine += s_seg[s];
        const uint32_t after = sel_suffix(mine, s_w);
        __shared__ uint32_t s_sum;
        if (tid == 0) s_sum = after;
        __syncthreads();
        uint32_t pre = s_sum - after;
        for (int s = s0; s < s1; ++s) {
            const uint32_t v = s_seg[s];
            s_seg[s] = (uint16_t)pre;
            pre += v;
        }
    }
    __syncthreads();
    VO_STAMP(d, 1960 + w, 8);
    // 5. each selected key at base + its segment's start + the selected keys before it in the segment
    const int slot = ext_slot(d, f0, z, slot_override);
    int2* out = d.kps + (size_t)slot * N;
    for (int g = tid; g < total; g += SL_T) {
        if (!((s_bits[g >> 6] >> (g & 63)) & 1ull)) continue;
        const int k = s_tof[g];
        const uint64_t key = key_of(g, k);
        const int row = (int)((key >> 16) & 0xFFFF), col = (int)(key & 0xFFFF);
        const int r = row & (ST_TH - 1);
        const uint4 rc = s_rows[k];
        const uint32_t w4[4] = {rc.x, rc.y, rc.z, rc.w};
        int start = s_pre[k];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int sh = 8 * min(max(r - 4 * q, 0), 4);
            const uint32_t msk = (uint32_t)(0xFFFFFFFFull >> (32 - sh));
            start = (int)__builtin_amdgcn_udot4(w4[q] & msk, 0x01010101u, (uint32_t)start, false);
        }
        int within = 0;
        for (int wi = start >> 6; wi <= (g >> 6); ++wi) {
            uint64_t m = s_bits[wi];
            if (wi == (start >> 6)) m &= ~0ull << (start & 63);
            if (wi == (g >> 6)) m &= (g & 63) ? (~0ull >> (64 - (g & 63))) : 0ull;
            within += __popcll(m);
        }
        const int pos = base + (int)s_seg[seg_of(key, k)] + within;
        if (pos < N) out[pos] = make_int2(col, row);
    }
    VO_STAMP(d, 1960 + w, 9);
}

__global__ void __launch_bounds__(SL_T) k_select_emit(VoDev d, int f0, int slot_override, int nb)
{
    int z, w;
    if (!xcd_frame(d, VO_SEL_BANDS, nb, z, w)) return;
    extern __shared__ __align__(16) unsigned char smem[];
    sel_emit_body(d, f0, slot_override, z, w, smem);
}

// The per-frame call's select: count and emit in one launch of the frame's VO_SEL_BANDS workgroups
// (one launch and one dependent-launch gap less than the two kernels).  The bands meet after the
// count: the last to arrive ranks the boundary keys and publishes ctl->ready (release, agent scope);
// every band waits for it (acquire) before emitting.  The launch follows its frame's stencil on the
// same queue, so its eight workgroups find the chip free and run together; the wait is bounded all
// the same -- a band that times out marks the frame VO_STATUS_INCONSISTENT and counts a device error
// instead of hanging -- and the last band to finish clears the flag for the next launch.
__global__ void __launch_bounds__(SL_T) k_select_fused(VoDev d, int f0, int slot_override, int nb)
{
    int z, w;
    if (!xcd_frame(d, VO_SEL_BANDS, nb, z, w)) return;
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ unsigned s_timeout, s_last2;
    VoSelCtl* ctl = d.selctl + z;
    const int ntx = (d.W + ST_TW - 1) / ST_TW, nty = (d.H + ST_TH - 1) / ST_TH;
    int total = 0, b = -1;
    // d.sel_fused == 2: bands of at most SL_TOF_CAP keys keep them in LDS and build the bitmap before
    // the wait (sel_emit_fused); 1 (VO_SEL_EARLY=0, or a frame whose fused LDS does not fit): the
    // emit after the wait (sel_emit_body)
    const bool early = d.sel_fused == 2;
    const bool last = sel_count_body(d, f0, slot_override, z, w, smem, true,
                                     early ? reinterpret_cast<uint64_t*>(smem + sel_fused_kbuf(ntx, nty)) : nullptr,
                                     &total, &b);
    __syncthreads();
    // wait for the last band's threshold and positions (the last band itself published them)
    auto wait = [&]() -> bool {
        if (!last) {
            if (threadIdx.x == 0) {
                unsigned it = 0u;
                // relaxed polls (a device-coherent load each), one acquire after the loop: an acquire poll
                // invalidates the XCD's L2 (buffer_inv sc1) on every iteration, under the working waves
                while (__hip_atomic_load((gu32*)&ctl->ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u &&
                       it < d.spin_limit) {
                    __builtin_amdgcn_s_sleep(2);
                    ++it;
                }
                s_timeout = it >= d.spin_limit ? 1u : 0u;
            }
            __syncthreads();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the ranked threshold and band positions
            if (s_timeout) {
                if (threadIdx.x == 0) {
                    const int slot = ext_slot(d, f0, z, slot_override);
                    d.ext_n[slot] = 0;
                    d.ext_st[slot] = VO_STATUS_INCONSISTENT;
                    atomicAdd(d.ctr + VO_CTR_ERR, 1u);
                    atomicOr(&ctl->timeout, 1u);   // the ranker may still store OK: re-marked below
                }
                return false;
            }
        } else {
            __syncthreads();
        }
        return true;
    };
    if (early && total <= SL_TOF_CAP) {
        sel_emit_fused(d, f0, slot_override, z, w, smem, total, b, wait);
    } else if (wait()) {
        sel_emit_body(d, f0, slot_override, z, w, smem);
    }
    if (!arrive_last(&ctl->arrive2, VO_SEL_BANDS, &s_last2)) return;
    if (threadIdx.x == 0) {
        // every band (the ranker included) has stored: a timed-out band's INCONSISTENT is final
        if (__hip_atomic_load((gu32*)&ctl->timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            const int slot = ext_slot(d, f0, z, slot_override);
            d.ext_n[slot] = 0;
            d.ext_st[slot] = VO_STATUS_INCONSISTENT;
            ctl->timeout = 0u;
        }
        ctl->ready = 0u; ctl->arrive2 = 0u;       // for the next launch
    }
}

// extract side of a missing image (VisualOdometry.cpp:77-82): the slot holds no keypoints
__global__ void k_ext_missing(VoDev d, int slot)
{
    if (threadIdx.x == 0) {
        d.ext_n[slot] = 0;
        d.ext_st[slot] = VO_STATUS_MISSING;
    }
}

// ---------------------------------------------------------------------------
// describe: orientation (903-term sequential f32 sums) + rotation + 512 tests.
// FREAK_feature_descriptor_parallel_GPU.cpp:10-210, kernels .c:124-225, orientation order
// FREAK_feature_descriptor_parallel.cpp:16-44.
// One wave per DS_KPW = 64 keypoints, lane = keypoint: a lane runs both 903-term sums of its
// keypoint itself, in order (one sample difference serves both components), reading its
// samples from its own LDS column; pair p's sample stays in a register over the pairs (p, q),
// the pair table arrives by scalar loads (the pair index is wave-uniform).  The term
// (ic*d)/|d| is fmaf(ic, A, ic * B) with the unit direction split into two f32 (equal to the f32
// division for every reachable ic and pair, tests/test_describe_division.py), so the sums use
// no f64.  The rotated samples stay in registers and the 512 tests, unrolled with the pattern's
// pair indices as compile-time constants, are register compares shifted into 32-bit words.
// No cross-lane traffic, no barrier.
// ---------------------------------------------------------------------------
#define DS_KPW 64
#ifndef DS_ALIGNBIT
#define DS_ALIGNBIT 1
#endif
#ifndef DS_WAVES
#define DS_WAVES 4
#endif
#define DS_KPB (DS_KPW * DS_WAVES)
#ifndef DS_PKSUB
#define DS_PKSUB 0             // 1: the orientation sums' sample differences two per v_pk_add_f32 (12 % fewer orientation VALU, but KITTI 288-290k vs 293-298k, r4s)
#endif
#ifndef DS_PROBE
#define DS_PROBE 0             // diagnostic builds only: 1 hot table, 2 no orientation sums (wrong descriptors)
#endif
#ifndef DS_UNROLL
#define DS_UNROLL 0            // 1: the orientation sums fully unrolled from sample registers (describe
                               // 0.92 -> 0.85 us/frame but KITTI 278-285k vs 283-289k: 110 VGPRs, 30 KB code)
#endif

// the FREAK lists of include/vo_freak_tables.h as compile-time tables; pair e is the e-th
// (p, q), p < q, row-major (ensure_tables enumerates the same order)
struct DsTables {
    int px[VO_FREAK_NPOINTS], py[VO_FREAK_NPOINTS];
    int patch[VO_FREAK_NTESTS];
    int pp[VO_FREAK_NPAIRS], pq[VO_FREAK_NPAIRS];
};
constexpr DsTables ds_make_tables()
{
    DsTables t{};
    constexpr int pts[VO_FREAK_NPOINTS][2] = {VO_FREAK_POINTS_LIST};
    constexpr short patch[VO_FREAK_NTESTS] = {VO_FREAK_PATCH_LIST};
    for (int i = 0; i < VO_FREAK_NPOINTS; ++i) { t.px[i] = pts[i][0]; t.py[i] = pts[i][1]; }
    for (int i = 0; i < VO_FREAK_NTESTS; ++i) t.patch[i] = patch[i];
    int e = 0;
    for (int p = 0; p < VO_FREAK_NPOINTS; ++p)
        for (int q = p + 1; q < VO_FREAK_NPOINTS; ++q) { t.pp[e] = p; t.pq[e] = q; ++e; }
    return t;
}
constexpr DsTables kDs = ds_make_tables();

// one orientation term of both components: (ic*dx)/|d|, (ic*dy)/|d| (c = Ax, Ay, Bx, By), the
// two components as one packed-FP32 pair (v_pk_mul/fma/add_f32: two lanes' worth per
// instruction, tools/valu_rate.hip; IEEE per element, so the sums are those of the scalar form)
typedef float ds_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void orient_term(float ic, const float4& c, ds_f2& o)
{
    const ds_f2 i2 = {ic, ic};
    o = o + __builtin_elementwise_fma(i2, ds_f2{c.x, c.y}, i2 * ds_f2{c.z, c.w});   // fmaf(ic, A, ic * B)
}

// the 32 tests 32 W .. 32 W + 31 of a keypoint's rotated samples r: bit i = test 32 W + i
template <int W>
__device__ __forceinline__ uint32_t ds_word(const uint32_t (&r)[VO_FREAK_NPOINTS])
{
    uint32_t word = 0u;
    st_for([&](auto J) {
        constexpr int t = 32 * W + 31 - decltype(J)::value;          // highest test first
        constexpr int e = kDs.patch[t];
#if DS_ALIGNBIT
        // (word << 1) | (I(q) - I(p) < 0): v_sub + v_alignbit_b32 (funnel shift of word:diff by 31),
        // no compare, no VCC select and its wait states (samples are bytes: no overflow)
        word = __builtin_amdgcn_alignbit(word, r[kDs.pq[e]] - r[kDs.pp[e]], 31u);
#else
        word = (word << 1) | (r[kDs.pp[e]] > r[kDs.pq[e]] ? 1u : 0u);
#endif
    }, std::make_integer_sequence<int, 32>{});
    return word;
}

// LT (diagnostic, VO_DS_LDS_TABLE=1 for the per-frame call): the orientation pair table read from an
// LDS copy instead of through the scalar cache.  Measured slower for a single frame too (26 -> 30 us),
// so the per-frame describe is not waiting on scalar-cache misses of the table.
template <bool LT>
__device__ __forceinline__ void describe_wave(const VoDev& d, const uint8_t* __restrict__ img, int cur, int n,
                                              int base, float (*s_I0)[DS_KPW], const float4* __restrict__ s_tab)
{
    constexpr int NP = VO_FREAK_NPOINTS;
    const int lane = threadIdx.x & 63;
    const int W = d.W, H = d.H, Wb = d.bstride;   // blurred plane: row stride Wb
    [[maybe_unused]] const int stamp_slot = 1000 + (int)((blockIdx.x * DS_WAVES + (threadIdx.x >> 6)) % 900);
    VO_STAMP(d, stamp_slot, 0);
    const bool valid = base + lane < n;
    // lanes past n sample around a keypoint inside the margin: every address stays in bounds
    // and the gathers need no branches (their values are never used)
    const int2 kp = valid ? d.kps[(size_t)cur * d.N + base + lane] : make_int2(d.bcol, d.brow);
    ds_f2 oxy = {0.0f, 0.0f};
#if DS_UNROLL
    // 1. the 43 pattern samples, in registers
    float smp[NP];
    {
        uint32_t v[NP];
        st_for([&](auto U) {
            constexpr int u = decltype(U)::value;
            v[u] = img[(size_t)(kp.y + kDs.py[u]) * Wb + (kp.x + kDs.px[u])];
        }, std::make_integer_sequence<int, NP>{});
        st_for([&](auto U) { smp[U] = (float)v[U]; }, std::make_integer_sequence<int, NP>{});
    }
    (void)s_I0;
    VO_STAMP(d, stamp_slot, 1);
    // 2. O = sum over pairs t = 0..902 of (ic * d) / |d|, each component in order in f32, fully
    //    unrolled: the pair (p, q) of term t is a compile-time constant, so ic = I(p) - I(q) reads
    //    two sample registers and the sums need no LDS, no padding terms and no loop control.  The
    //    table arrives by scalar loads, one block of DS_UB entries ahead of the block being summed.
    {
        constexpr int NB = (VO_FREAK_NPAIRS + DS_UB - 1) / DS_UB;
        float4 tb[DS_UB], tbn[DS_UB];
#pragma unroll
        for (int u = 0; u < DS_UB; ++u) tb[u] = c_orient_u[u];
        st_for([&](auto Bk) {
            constexpr int b = decltype(Bk)::value;
            // block b's entries (requested during block b - 1) have arrived; request block b + 1
            __builtin_amdgcn_s_waitcnt(0xC07F);         // lgkmcnt(0)
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (b + 1 < NB) {
#pragma unroll
                for (int u = 0; u < DS_UB; ++u) tbn[u] = c_orient_u[(b + 1) * DS_UB + u];
            }
            __builtin_amdgcn_sched_barrier(0);          // the requests stay ahead of the sums
            st_for([&](auto U) {
                constexpr int t = b * DS_UB + decltype(U)::value;
                if constexpr (t < VO_FREAK_NPAIRS) orient_term(smp[kDs.pp[t]] - smp[kDs.pq[t]], tb[U], oxy);
            }, std::make_integer_sequence<int, DS_UB>{});
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (b + 1 < NB) {
#pragma unroll
                for (int u = 0; u < DS_UB; ++u) tb[u] = tbn[u];
            }
        }, std::make_integer_sequence<int, NB>{});
    }
#else
    // 1. the 43 pattern samples -> this lane's LDS column (all loads in flight first)
    {
        uint32_t v[NP];
        st_for([&](auto U) {
            constexpr int u = decltype(U)::value;
            v[u] = img[(size_t)(kp.y + kDs.py[u]) * Wb + (kp.x + kDs.px[u])];
        }, std::make_integer_sequence<int, NP>{});
        st_for([&](auto U) { s_I0[U][lane] = (float)v[U]; }, std::make_integer_sequence<int, NP>{});
#pragma unroll
        for (int u = NP; u < DS_OROWS; ++u) s_I0[u][lane] = 0.0f;     // the padding terms' samples
    }
    VO_STAMP(d, stamp_slot, 1);
    // 2. O = sum over pairs t = 0..902 of (ic * d) / |d|, each component in order in f32; row p
    //    (pairs (p, q), q > p) in groups of DS_OG, the last one padded with zero terms that read
    //    the zero rows past the samples.  Software-pipelined: the samples and table entries of
    //    group g + 1 are requested before group g is summed.
    {
#if DS_PROBE == 2
        constexpr int NG = 1;                           // probe: no orientation sums
#else
        constexpr int NG = DS_ONPAD / DS_OG;
#endif
        const float* col = &s_I0[0][lane];
        int p = 0, qs = 1;                              // group g: row p, samples qs .. qs + 7
        float ip = col[0], iq[DS_OG];
        float4 tb[DS_OG];
#pragma unroll
        for (int u = 0; u < DS_OG; ++u) { iq[u] = col[(qs + u) * DS_KPW]; tb[u] = LT ? s_tab[u] : c_orient[u]; }
#ifndef DS_GUNROLL
#define DS_GUNROLL 4          // orientation groups unrolled (2: 269k vs 277k frames/s in alternating A/B)
#endif
#pragma unroll DS_GUNROLL
        for (int g = 0; g < NG; ++g) {
            // the next group (the last one re-reads itself)
            int pn = p, qn = qs + DS_OG;
            if (qn >= VO_FREAK_NPOINTS) { pn = p + 1; qn = p + 2; }
            const int gn = g + 1 < NG ? g + 1 : g;
            if (g + 1 >= NG) { pn = p; qn = qs; }
            // group g's samples and table entries (requested during group g - 1) have arrived:
            // wait here, before the next requests, since a scalar load in flight makes any
            // LDS wait a wait for everything
            __builtin_amdgcn_s_waitcnt(0xC07F);         // lgkmcnt(0)
            __builtin_amdgcn_sched_barrier(0);
            const float ipn = col[pn * DS_KPW];
            float iqn[DS_OG];
            float4 tbn[DS_OG];
#pragma unroll
            for (int u = 0; u < DS_OG; ++u) {
#if DS_PROBE == 1
                iqn[u] = col[(qn + u) * DS_KPW]; tbn[u] = c_orient[(gn & 3) * DS_OG + u];   // probe: a hot 512-byte table
#else
                iqn[u] = col[(qn + u) * DS_KPW]; tbn[u] = LT ? s_tab[gn * DS_OG + u] : c_orient[gn * DS_OG + u];
#endif
            }
            __builtin_amdgcn_sched_barrier(0);          // the requests stay ahead of the sums
#pragma unroll
#if DS_PKSUB
            // two sample differences per packed subtract (exact: integers), each broadcast into
            // its term's packed product by op_sel
            for (int u = 0; u < DS_OG; u += 2) {
                static_assert(DS_OG % 2 == 0, "pairs of terms");
                const ds_f2 dd = ds_f2{ip, ip} - ds_f2{iq[u], iq[u + 1]};
                orient_term(dd.x, tb[u], oxy);
                orient_term(dd.y, tb[u + 1], oxy);
            }
#else
            for (int u = 0; u < DS_OG; ++u) orient_term(ip - iq[u], tb[u], oxy);
#endif
            __builtin_amdgcn_sched_barrier(0);
            p = pn; qs = qn; ip = ipn;
#pragma unroll
            for (int u = 0; u < DS_OG; ++u) { iq[u] = iqn[u]; tb[u] = tbn[u]; }
        }
    }
#endif
    VO_STAMP(d, stamp_slot, 2);
    const float ox = oxy.x, oy = oxy.y;
    // 3. angle and rotation
    float angle = 0.0f;
    if (!(isnan(ox) || isnan(oy))) angle = (float)det_atan2((double)oy, (double)ox);
    double sd, cd;
    det_sincos((double)angle, &sd, &cd);
    const float c = (float)cd, s = (float)sd, ms = -1.0f * s;
    VO_STAMP(d, stamp_slot, 3);
    // 4. rotated samples (quirk 4: A = [[c, s], [s, c]], (int) truncation), in registers
    uint32_t r[NP];
    st_for([&](auto U) {
        constexpr int u = decltype(U)::value, px = kDs.px[u], py = kDs.py[u];
        int x = (int)(((float)kp.x + (float)px * c) + (float)py * s);
        int y = (int)(((float)kp.y + (float)(-1 * px) * ms) + (float)py * c);
        x = min(max(x, 0), W - 1);   // in range for every keypoint inside the margin
        y = min(max(y, 0), H - 1);
        r[u] = img[(size_t)y * Wb + x];
    }, std::make_integer_sequence<int, NP>{});
    VO_STAMP(d, stamp_slot, 4);
    // 5. the 512 tests: 16 words of 32, stored as the 8 u64 of the packed descriptor
    uint32_t w[16];
    w[0] = ds_word<0>(r);   w[1] = ds_word<1>(r);   w[2] = ds_word<2>(r);   w[3] = ds_word<3>(r);
    w[4] = ds_word<4>(r);   w[5] = ds_word<5>(r);   w[6] = ds_word<6>(r);   w[7] = ds_word<7>(r);
    w[8] = ds_word<8>(r);   w[9] = ds_word<9>(r);   w[10] = ds_word<10>(r); w[11] = ds_word<11>(r);
    w[12] = ds_word<12>(r); w[13] = ds_word<13>(r); w[14] = ds_word<14>(r); w[15] = ds_word<15>(r);
    if (valid) {
        uint4* dst = reinterpret_cast<uint4*>(d.desc + ((size_t)cur * d.N + base + lane) * 8);
        dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
        dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
        dst[2] = make_uint4(w[8], w[9], w[10], w[11]);
        dst[3] = make_uint4(w[12], w[13], w[14], w[15]);
        d.pre[(size_t)cur * d.N + base + lane] = w[0];
    }
    VO_STAMP(d, stamp_slot, 5);
}

// grid xcd_grid(N / DS_KPB, nb) (frame z of the batch, workgroup bx of the frame, xcd_frame).
// publish > 0: the last workgroup of the launch tells the pose queue that frames < publish are
// extracted (every workgroup of the grid arrives, padding included)
template <bool LT>
__global__ void __launch_bounds__(64 * DS_WAVES) k_describe(VoDev d, int f0, int slot_override, unsigned publish,
                                                            int nb)
{
    __shared__ float s_I0[DS_WAVES][DS_UNROLL ? 1 : DS_OROWS][DS_KPW];   // sample columns (the looped sums)
    __shared__ float4 s_tab[LT ? DS_ONPAD : 1];                          // LT: the pair table
    if constexpr (LT) {
        for (int i = threadIdx.x; i < DS_ONPAD; i += 64 * DS_WAVES) s_tab[i] = c_orient[i];
        __syncthreads();
    }
#if LDS_POISON
    {
        const uint32_t pz = (uint32_t)wall_clock64() * 0x9E3779B9u ^ (uint32_t)blockIdx.x;
        float* w = &s_I0[0][0][0];
        for (int i = threadIdx.x; i < (int)(sizeof(s_I0) / 4); i += 64 * DS_WAVES) w[i] = __uint_as_float(pz + (uint32_t)i);
        __syncthreads();
    }
#endif
    int z, bx;
    if (xcd_frame(d, (d.N + DS_KPB - 1) / DS_KPB, nb, z, bx)) {
        const int cur = ext_slot(d, f0, z, slot_override);
        const int n = d.ext_n[cur];
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const int base = bx * DS_KPB + wave * DS_KPW;
        if (base < n)                    // wave-uniform; no barrier inside
            describe_wave<LT>(d, d.blurred + (size_t)z * d.bplane + VO_BLUR_X0, cur, n, base, s_I0[wave], s_tab);
    }
    if (!publish) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __shared__ unsigned s_last;
    if (!arrive_last(d.ctr + VO_CTR_DESCRIBE + 16 * d.eq, gridDim.x, &s_last)) return;
    if (threadIdx.x == 0) d.ctr[VO_CTR_DESCRIBE + 16 * d.eq] = 0u;
    publish_seq(d.ctr + VO_SYNC_EXT + 16 * d.eq, publish);
}

// ---------------------------------------------------------------------------
// The per-frame call's describe (k_describe_pf): one 64-keypoint block per workgroup of DP_WAVES
// waves instead of one wave, lane = keypoint as in describe_wave, the same arithmetic in the same
// order.  One wave alone walks 43 gathers, 903 in-order terms, 43 rotated gathers and 512 tests per
// keypoint -- the per-frame call's longest link (26.5 us).  Here the waves share every phase but
// the in-order sum: the pattern and rotated gathers (a sample row per wave in turn, into LDS), the
// orientation terms (fmaf(ic, A, ic * B) per component, exactly describe_wave's term) computed a
// chunk ahead into an LDS ring by waves 1.., while wave 0 adds each chunk's terms to the running
// f32 sums in pair order t = 0 .. 902 (so every rounding is the sequential loop's), and the 16
// test words (two per wave).
// ---------------------------------------------------------------------------
// pair (p, q) of orientation term t, p < q in the pattern's pair order (compile-time: the term
// waves of k_describe_pf generate one straight-line block per term)
__host__ __device__ constexpr int dp_pair_p(int t)
{
    int p = 0;
    for (int cnt = VO_FREAK_NPOINTS - 1; t >= cnt; --cnt) { t -= cnt; ++p; }
    return p;
}
__host__ __device__ constexpr int dp_pair_q(int t)
{
    int p = 0, cnt = VO_FREAK_NPOINTS - 1;
    for (; t >= cnt; --cnt) { t -= cnt; ++p; }
    return p + 1 + t;
}
static_assert(dp_pair_p(0) == 0 && dp_pair_q(0) == 1 && dp_pair_p(42) == 1 && dp_pair_q(42) == 2, "pair order");
#define DP_WAVES 8
#ifndef DP_CT_TERMS
#define DP_CT_TERMS 1                  // term waves with compile-time pairs and samples in registers
#endif
#define DP_CH DP_CHUNK                               // terms per chunk of the LDS ring (two chunks)
// k_describe_pf's term wave W (1 .. DP_WAVES - 1): the terms t = W - 1 (mod DP_WAVES - 1) of each
// chunk, generated at compile time (pairs as register indices into the wave's 43 samples, weights by
// scalar loads at fixed offsets), a barrier after each chunk as the sum wave expects
template <int W, int T, int J>
__device__ __forceinline__ void dp_one_term(const float* I, ds_f2 (*slot)[64], int lane)
{
    if constexpr (T < VO_FREAK_NPAIRS && T % (DP_WAVES - 1) == W - 1) {
        constexpr int P = dp_pair_p(T), Q = dp_pair_q(T);
        const float4 tb = c_orient_u[T];
        const float ic = I[P] - I[Q];
        const ds_f2 i2 = {ic, ic};
        slot[J][lane] = __builtin_elementwise_fma(i2, ds_f2{tb.x, tb.y}, i2 * ds_f2{tb.z, tb.w});
    }
}
template <int W, int C, int... J>
__device__ __forceinline__ void dp_chunk_terms(const float* I, ds_f2 (*slot)[64], int lane, std::integer_sequence<int, J...>)
{
    (dp_one_term<W, C * DP_CH + J, J>(I, slot, lane), ...);
}
template <int W, int... C>
__device__ __forceinline__ void dp_term_wave(const float* I, ds_f2 (*s_t)[DP_CH + 1][64], int lane,
                                             std::integer_sequence<int, C...>)
{
    ((dp_chunk_terms<W, C>(I, s_t[C & 1], lane, std::make_integer_sequence<int, DP_CH>{}), __syncthreads()), ...);
    __syncthreads();                                 // the sum wave's last chunk
}
__global__ void __launch_bounds__(64 * DP_WAVES) k_describe_pf(VoDev d, int f0, int slot_override)
{
    constexpr int NP = VO_FREAK_NPOINTS;
    constexpr int NC = (VO_FREAK_NPAIRS + DP_CH - 1) / DP_CH;
    __shared__ float s_I[NP][64];                    // pattern samples (then the rotated samples, as u32)
    __shared__ ds_f2 s_t[2][DP_CH + 1][64];          // orientation terms, a chunk ahead (+ a spare row)
    __shared__ float s_c[64], s_s[64];
#if !DP_CT_TERMS
    __shared__ float4 s_orient[DP_NPAD];
    __shared__ uint32_t s_pairoff[DP_NPAD];
#endif
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int cur = ext_slot(d, f0, 0, slot_override);
    const int n = d.ext_n[cur];
    const int base = blockIdx.x * 64;
    if (base >= n) return;                           // workgroup-uniform
    const int W = d.W, H = d.H, Wb = d.bstride;
    const uint8_t* __restrict__ img = d.blurred + VO_BLUR_X0;
    [[maybe_unused]] const int sslot = 1000 + blockIdx.x * DP_WAVES + wave;
    VO_STAMP(d, sslot, 0);
    const bool valid = base + lane < n;
    const int2 kp = valid ? d.kps[(size_t)cur * d.N + base + lane] : make_int2(d.bcol, d.brow);
#if !DP_CT_TERMS
    // 0. the term tables into LDS
    for (int t = threadIdx.x; t < DP_NPAD; t += 64 * DP_WAVES) {
        s_orient[t] = c_orient_pf[t];
        s_pairoff[t] = c_pairoff[t];
    }
#endif
    // 1. pattern samples, rows u = wave, wave + DP_WAVES, ...
    for (int u = wave; u < NP; u += DP_WAVES)
        s_I[u][lane] = (float)img[(size_t)(kp.y + (int)c_ppt[u].y) * Wb + (kp.x + (int)c_ppt[u].x)];
    __syncthreads();
    VO_STAMP(d, sslot, 1);
    // 2. terms of chunk c into ring slot c & 1 by waves 1 .. DP_WAVES - 1 (term t of the chunk by wave
    //    1 + t % (DP_WAVES - 1)); wave 0 sums chunk c - 1 meanwhile
    //    A wave's terms of a chunk are a fixed unrolled run (j = wave - 1 + 7 i) over the padded
    //    tables, so its scalar loads and LDS reads are all in flight at once (the loop with a
    //    data-dependent exit and a byte table in global memory left wave 0 waiting at every chunk
    //    barrier: 47k of the wave's 62k cycles)
    //    The tables come from LDS (copied at entry): scalar loads share lgkmcnt with the LDS
    //    reads, so every term waited for its scalar load's full latency (54k cycles at wave 0)
#if !DP_CT_TERMS
    static_assert(DP_CH == DP_CHUNK, "k_describe_pf's chunk is its tables' padding unit");
    const unsigned char* sIb = reinterpret_cast<const unsigned char*>(&s_I[0][0]) + 4 * lane;
    auto terms = [&](int c) {
        constexpr int TPW = (DP_CH + DP_WAVES - 2) / (DP_WAVES - 1);
        // branch-free (a wave's run past the chunk writes the spare row DP_CH), so the compiler
        // issues the run's LDS reads together instead of three dependent round trips per term
        // (in three sweeps -- the run's pair offsets, then its samples and weights, then the terms
        // -- so each sweep's reads are in flight together)
        uint32_t po[TPW];
        float4 tb[TPW];
        float ia[TPW], ib[TPW];
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int t = c * DP_CH + min(wave - 1 + (DP_WAVES - 1) * i, DP_CH - 1);
            po[i] = s_pairoff[t];
            tb[i] = s_orient[t];
        }
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            ia[i] = *reinterpret_cast<const float*>(sIb + (po[i] & 0xFFFFu));
            ib[i] = *reinterpret_cast<const float*>(sIb + (po[i] >> 16));
        }
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int j = min(wave - 1 + (DP_WAVES - 1) * i, DP_CH);
            const float ic = ia[i] - ib[i];
            const ds_f2 i2 = {ic, ic};
            s_t[c & 1][j][lane] = __builtin_elementwise_fma(i2, ds_f2{tb[i].x, tb[i].y}, i2 * ds_f2{tb[i].z, tb[i].w});
        }
    };
#endif
    ds_f2 oxy = {0.0f, 0.0f};
#if DP_CT_TERMS
    // term wave W (1 .. DP_WAVES - 1) computes the terms t = W - 1 (mod DP_WAVES - 1) with
    // compile-time pairs: its 43 samples in registers, the weights by scalar loads, no table or
    // sample reads through LDS (those made the term waves LDS-bound: 25-29k cycles per block)
    float I[NP];
    if (wave > 0) {
#pragma unroll
        for (int u = 0; u < NP; ++u) I[u] = s_I[u][lane];
    }
    switch (wave) {
    case 0: {
        __syncthreads();                             // chunk 0 written
        for (int c = 0; c < NC; ++c) {
            const int m = min(DP_CH, VO_FREAK_NPAIRS - c * DP_CH);
#pragma unroll 16
            for (int j = 0; j < m; ++j) oxy = oxy + s_t[c & 1][j][lane];
            __syncthreads();
        }
        break;
    }
    case 1: dp_term_wave<1>(I, s_t, lane, std::make_integer_sequence<int, NC>{}); break;
    case 2: dp_term_wave<2>(I, s_t, lane, std::make_integer_sequence<int, NC>{}); break;
    case 3: dp_term_wave<3>(I, s_t, lane, std::make_integer_sequence<int, NC>{}); break;
    case 4: dp_term_wave<4>(I, s_t, lane, std::make_integer_sequence<int, NC>{}); break;
    case 5: dp_term_wave<5>(I, s_t, lane, std::make_integer_sequence<int, NC>{}); break;
    case 6: dp_term_wave<6>(I, s_t, lane, std::make_integer_sequence<int, NC>{}); break;
    default: dp_term_wave<7>(I, s_t, lane, std::make_integer_sequence<int, NC>{}); break;
    }
#else
    if (wave > 0) terms(0);
    __syncthreads();
    for (int c = 0; c < NC; ++c) {
        if (wave > 0) {
            if (c + 1 < NC) terms(c + 1);
        } else {
            const int m = min(DP_CH, VO_FREAK_NPAIRS - c * DP_CH);
#pragma unroll 16
            for (int j = 0; j < m; ++j) oxy = oxy + s_t[c & 1][j][lane];
        }
        __syncthreads();
    }
#endif
    VO_STAMP(d, sslot, 2);
    // 3. angle and rotation (wave 0), as describe_wave
    if (wave == 0) {
        const float ox = oxy.x, oy = oxy.y;
        float angle = 0.0f;
        if (!(isnan(ox) || isnan(oy))) angle = (float)det_atan2((double)oy, (double)ox);
        double sd, cd;
        det_sincos((double)angle, &sd, &cd);
        s_c[lane] = (float)cd;
        s_s[lane] = (float)sd;
    }
    __syncthreads();
    VO_STAMP(d, sslot, 3);
    // 4. rotated samples (quirk 4), rows u = wave, wave + DP_WAVES, ...
    {
        const float c = s_c[lane], s = s_s[lane], ms = -1.0f * s;
        uint32_t* rot = reinterpret_cast<uint32_t*>(&s_I[0][0]);
        for (int u = wave; u < NP; u += DP_WAVES) {
            const int px = c_ppt[u].x, py = c_ppt[u].y;
            int x = (int)(((float)kp.x + (float)px * c) + (float)py * s);
            int y = (int)(((float)kp.y + (float)(-1 * px) * ms) + (float)py * c);
            x = min(max(x, 0), W - 1);
            y = min(max(y, 0), H - 1);
            rot[u * 64 + lane] = img[(size_t)y * Wb + x];
        }
    }
    __syncthreads();
    VO_STAMP(d, sslot, 4);
    // 5. the 512 tests: words wave and wave + 8 of 16
    {
        const uint32_t* rot = reinterpret_cast<const uint32_t*>(&s_I[0][0]);
        uint32_t r[NP];
#pragma unroll
        for (int u = 0; u < NP; ++u) r[u] = rot[u * 64 + lane];
        uint32_t w0 = 0u, w1 = 0u;
        switch (wave) {
        case 0: w0 = ds_word<0>(r); w1 = ds_word<8>(r); break;
        case 1: w0 = ds_word<1>(r); w1 = ds_word<9>(r); break;
        case 2: w0 = ds_word<2>(r); w1 = ds_word<10>(r); break;
        case 3: w0 = ds_word<3>(r); w1 = ds_word<11>(r); break;
        case 4: w0 = ds_word<4>(r); w1 = ds_word<12>(r); break;
        case 5: w0 = ds_word<5>(r); w1 = ds_word<13>(r); break;
        case 6: w0 = ds_word<6>(r); w1 = ds_word<14>(r); break;
        default: w0 = ds_word<7>(r); w1 = ds_word<15>(r); break;
        }
        if (valid) {
            uint32_t* dst = reinterpret_cast<uint32_t*>(d.desc + ((size_t)cur * d.N + base + lane) * 8);
            dst[wave] = w0;
            dst[wave + 8] = w1;
            if (wave == 0) d.pre[(size_t)cur * d.N + base + lane] = w0;
        }
    }
    VO_STAMP(d, sslot, 5);
}

// ---------------------------------------------------------------------------
// match: brute-force Hamming top-2 + Lowe ratio, one query per wave; the last workgroup
// compacts the accepted queries in ascending order into matches + f64 points.
// feature_matching_parallel.cpp:39-113; VisualOdometry.cpp:100-123.
// key = dist<<16 | j, so the min key is (min dist, first j) and the 2nd key gives `second`
// ---------------------------------------------------------------------------
// branch-free top-2 update (keys are unique: the low 16 bits carry the candidate index)
__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c)
{
    return max(min(a, b), min(max(a, b), c));     // selected as v_med3_u32
}
// (m1 <= m2 always: the new second smallest is the median of key, m1, m2 -- one v_med3_u32)
__device__ __forceinline__ void top2_insert(uint32_t key, uint32_t& m1, uint32_t& m2)
{
    m2 = med3_u32(key, m1, m2);
    m1 = min(m1, key);
}
// two keys at once (m1 <= m2): the smallest of the four is min3(m1, k1, k2); the second
// smallest is the median of {m1, k1, k2} unless m2 is below it -- three VALU for two keys
// (v_med3_u32, v_min_u32, v_min3_u32) instead of four
__device__ __forceinline__ void top2_insert2(uint32_t k1, uint32_t k2, uint32_t& m1, uint32_t& m2)
{
    m2 = min(med3_u32(m1, k1, k2), m2);
    uint32_t r;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(m1), "v"(k1), "v"(k2));   // left alone, LLVM emits two v_min_u32
    m1 = r;
}
__device__ __forceinline__ void top2_wave(uint32_t& m1, uint32_t& m2)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        uint32_t o1 = __shfl_xor(m1, off), o2 = __shfl_xor(m2, off);
        uint32_t n1v = min(m1, o1);
        uint32_t n2v = min(max(m1, o1), min(m2, o2));
        m1 = n1v; m2 = n2v;
    }
}
// Lowe ratio test on the top-2 keys (feature_matching_parallel.cpp:90-99); needs 2 candidates
__device__ __forceinline__ int ratio_accept(uint32_t m1, uint32_t m2, float ratio)
{
    if (m1 == 0xFFFFFFFFu || m2 == 0xFFFFFFFFu) return -1;
    int d1 = (int)(m1 >> 16), d2 = (int)(m2 >> 16);
    return ((float)d1 < ratio * (float)d2) ? (int)(m1 & 0xFFFF) : -1;
}

// 32-bit prefix mode: MT_QPL queries per lane, 64 MT_QPL per workgroup (k_match)
#ifndef MT_QPL
#define MT_QPL 4
#endif
#define MT_QPB (64 * MT_QPL)
#ifndef MT_SINGLE_WAVES
#define MT_SINGLE_WAVES 16            // single-frame calls: waves per 64 queries (each walks 1/16 of the candidates)
#endif
#define MT512_QPB 256                 // 512-test matcher: queries per workgroup (one per thread)
__host__ __device__ inline int match_blocks(int N, int match_bits)
{
    return match_bits == 32 ? (N + MT_QPB - 1) / MT_QPB : (N + MT512_QPB - 1) / MT512_QPB;
}

// Window of a pose pass: frames [lo, lo + n), n = min(win, d.gmax - lo) (gmax <= the frames enqueued) with
// win <= d.WB: up to WB frames (2 extract batches), but only frames the pass's extract wait
// covers (d.gmax), so the window grows when the pose queue lags behind the extract queue and each
// pass's fixed latency is spread over more frames.  win is WB, or d.repair_win after a pass whose
// commit stopped early: the frames after a speculation miss (a frame that did not advance desc1)
// are re-run in a short window, since misses come in runs (a new sequence's first frames without
// a model, quirk 9) and each re-run window commits only up to the next miss.
// k_match decides the window (pass_window, every workgroup alike) and its first workgroup
// records it (d.plan); the pass's later kernels read the record (pass_plan).  With cross-pass
// pipelining (vo_internal.h VoPlan) the window comes from the state after pass p - 2 and pass
// p - 1's window; d.nospec (every earlier pass finalized) takes it from the state itself.
__device__ __forceinline__ VoPlan pass_window(const VoDev& d)
{
    const VoState* st = d.st;
    VoPlan P;
    int win;
    if (d.nospec) {
        P.lo = st->lo; P.dual = st->dual; P.prev0 = st->prev_slot; win = st->win;
    } else {
        const VoSnap s = d.snap[(d.pass + VO_PASS_RING - 2) & (VO_PASS_RING - 1)];
        const VoPlan q = d.plan[(d.pass + VO_PASS_RING - 1) & (VO_PASS_RING - 1)];
        if (q.n > 0 && q.lo == s.lo && q.prev0 == s.prev_slot) {
            // pass p - 1 starts where pass p - 2 left off: speculate that it commits its window
            P.lo = q.lo + q.n; P.dual = 0; P.prev0 = (P.lo - 1) % VO_RING; win = d.WB;
        } else {
            // pass p - 1 will be discarded (or commits nothing): the state after pass p - 2 holds
            P.lo = s.lo; P.dual = s.dual; P.prev0 = s.prev_slot; win = s.win;
        }
    }
    P.n = max(0, min(d.gmax - P.lo, win > 0 && win < d.WB ? win : d.WB));
    return P;
}
__device__ __forceinline__ VoPlan pass_plan(const VoDev& d) { return d.plan[d.pass & (VO_PASS_RING - 1)]; }
__device__ __forceinline__ int win_count(const VoDev& d, int stage)
{
    return stage ? 1 : pass_plan(d).n;
}
// Work records of a pass: one per window frame, and in a repair window (plan.dual) a second
// set [n, 2n): frame wf matched against desc1 as it was before the window (plan.prev0)
// instead of frame f - 1.  When frame f - 1 does not advance desc1 and no frame of the window
// before it did, that is the match the sequential loop makes, so a run of frames without a
// model (a new sequence's first frames) commits in one repair pass (k_finalize picks the
// record per frame).  repair_win <= WB / 2.
__device__ __forceinline__ int vwin_records(const VoPlan& P) { return P.dual ? 2 * P.n : P.n; }
__device__ __forceinline__ int vwin_count(const VoDev& d, int stage)
{
    if (stage) return 1;
    return vwin_records(pass_plan(d));
}
// k_match's window: decided here, recorded by the first workgroup for the pass's later kernels
__device__ __forceinline__ VoPlan match_window(const VoDev& d, int stage)
{
    if (stage) return VoPlan{0, 1, 0, 0};
    const VoPlan P = pass_window(d);
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) d.plan[d.pass & (VO_PASS_RING - 1)] = P;
    return P;
}

__device__ __forceinline__ uint64_t frame_seed_of(const VoDev& d, int f)
{
    return mix64(d.seed + 0x632BE59BD9B4E019ULL * (uint64_t)(f + 1));
}

// First frame (since vo_reset) of the sequence holding frame f: 0, or the largest of the sorted
// vo_set_sequence_starts entries <= f (binary search; block-uniform).  A frame is its sequence's
// frame f - base: the FIRST status and the RANSAC sampler's frame index follow it.
__device__ __forceinline__ int seq_base(const VoDev& d, int f)
{
    int lo = 0, hi = d.n_seq_starts;               // first entry > f
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (d.seq_starts[mid] <= f) lo = mid + 1; else hi = mid;
    }
    return lo > 0 ? d.seq_starts[lo - 1] : 0;
}

// Header of a window frame's match: slots and status (speculation: the previous frame of
// window frame wf > 0 is frame f - 1; k_finalize re-runs f when that was skipped).  Block 0
// initialises the frame's VoWork.  Returns false if the frame has nothing to match.
struct MatchFrame {
    VoWork* w;
    int f, cur, prev, n1, n2;
    int32_t* match_j;
};
__device__ __forceinline__ bool match_header(const VoDev& d, int stage, const VoPlan& P, int wf, MatchFrame& m)
{
    VoWork* w = d.work + wf;
    int f, fl = -1, cur, prev, status = VO_STATUS_OK;
    if (stage) {
        f = -1; prev = VO_STAGE_SLOT; cur = VO_STAGE_SLOT + 1;
    } else {
        const int n = P.n, df = wf < n ? wf : wf - n;   // record wf >= n: the dual match
        f = P.lo + df;
        cur = f % VO_RING;
        prev = df == 0 || wf >= n ? P.prev0 : (f - 1) % VO_RING;
        const int es = d.ext_st[cur];
        const int base = seq_base(d, f);
        fl = f - base;
        if (fl == 0) status = VO_STATUS_FIRST;                 // VisualOdometry.cpp:58,64-66
        else if (es != VO_STATUS_OK) status = es;              // MISSING / INCONSISTENT
        if (base == 0) fl += d.origin;                         // a sequence shard: the sampler's frame index
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        w->frame = f; w->cur = cur; w->prev = prev;
        w->bestk = -1; w->n_eval = 0; w->n_inl = 0; w->fitted = 0; w->n_fit = 0; w->degenerate = 0;
        w->need_more = 0;
        w->ready1 = 0u;                                        // k_ransac_fused's hand-off flag
        // the RANSAC chunks' arrival counters (each chunk's last arriver clears its own; a timed-out
        // fused wait leaves one short)
        w->ctr[1] = 0u; w->ctr[2] = 0u; w->ctr[3] = 0u;
        for (int c = 0; c < 4; ++c) w->counts4[c] = 0;
        if (!stage) w->frame_seed = frame_seed_of(d, fl);
        if (status != VO_STATUS_OK) { w->status = status; w->M = 0; w->scored = 0; }
    }
    m.w = w; m.f = f; m.cur = cur; m.prev = prev;
    m.n1 = d.ext_n[prev];
    m.n2 = d.ext_n[cur];
    m.match_j = d.match_j + (size_t)wf * d.N;
    return status == VO_STATUS_OK;
}

// The frame's last workgroup (its first 256 threads): ordered compaction of the accepted queries into
// (prev, cur) pairs and f64 points, thread t owning queries [t*per, (t+1)*per); M, scored and
// the < 8 matches status (VisualOdometry.cpp:108-123).
__device__ void match_compact(const VoDev& d, int wf, const MatchFrame& m, int* s_wsum)
{
    // rounds of 256 queries (thread t: query 256 u + t), in order: a match's position is the
    // matches of the earlier rounds, of the earlier waves of its round, and of the lower lanes
    // of its wave (ballot counts, one barrier per 8 rounds)
    constexpr int RC = 8;                         // rounds per pass (s_wsum holds RC x 4 counts)
    const int N = d.N, n1 = m.n1, lane = threadIdx.x & 63;
    const int tid = threadIdx.x, wave = tid >> 6;
    const bool act = tid < 256;                   // wider workgroups: the extra waves only meet the barriers
    const int2* kp1 = d.kps + (size_t)m.prev * N;
    const int2* kp2 = d.kps + (size_t)m.cur * N;
    int2* match_pairs = d.match_pairs + (size_t)wf * N;
    double* pts = d.pts + (size_t)wf * 4 * N;
    float* pts32 = d.pts32 + (size_t)wf * VO_PTS32_PER(N);
    VO_STAMP(d, 1993, 2);
    int pos0 = 0;                                 // matches of the earlier passes
    for (int r0 = 0; r0 * 256 < n1; r0 += RC) {
        int js[RC];
#pragma unroll
        for (int u = 0; u < RC; ++u) {
            const int i = (r0 + u) * 256 + tid;
            js[u] = act && i < n1 ? ld_sc1(m.match_j + i) : -1;
        }
        int2 ka[RC], kb[RC];
#pragma unroll
        for (int u = 0; u < RC; ++u) {
            ka[u] = make_int2(0, 0); kb[u] = make_int2(0, 0);
            if (js[u] >= 0) { ka[u] = kp1[(r0 + u) * 256 + tid]; kb[u] = kp2[js[u]]; }
        }
        unsigned long long bal[RC];
#pragma unroll
        for (int u = 0; u < RC; ++u) {
            bal[u] = ballot64(js[u] >= 0);
            if (lane == 0 && act) s_wsum[u * 4 + wave] = __popcll(bal[u]);
        }
        __syncthreads();
        int pos = pos0;
#pragma unroll
        for (int u = 0; u < RC; ++u) {
            int before = 0, total = 0;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const int c = s_wsum[u * 4 + w];
                before += w < wave ? c : 0;
                total += c;
            }
            if (js[u] >= 0) {
                const int p = pos + before + __popcll(bal[u] & ((1ull << lane) - 1ull));
                match_pairs[p] = make_int2((r0 + u) * 256 + tid, js[u]);
                const int2 a = ka[u], b = kb[u];
                double2* pp = reinterpret_cast<double2*>(pts + 4 * (size_t)p);
                pp[0] = make_double2((double)a.x, (double)a.y);
                pp[1] = make_double2((double)b.x, (double)b.y);
                pts32[vo_pts32_index(p, 0)] = (float)a.x;        // exact: pixel coordinates
                pts32[vo_pts32_index(p, 1)] = (float)a.y;
                pts32[vo_pts32_index(p, 2)] = (float)b.x;
                pts32[vo_pts32_index(p, 3)] = (float)b.y;
            }
            pos += total;
        }
        pos0 = pos;
        __syncthreads();                          // s_wsum is rewritten by the next pass
    }
    if (tid == 0) {
        VoWork* w = m.w;
        const int M = pos0;
        w->M = M;
        w->scored = (M / d.T) * d.T;
        w->status = M < 8 ? VO_STATUS_FEW_MATCHES : VO_STATUS_OK;   // VisualOdometry.cpp:108-115
        w->ctr[0] = 0u;
        w->cmax[0] = (float)d.W; w->cmax[1] = (float)d.H;        // keypoints lie inside the frame
        w->cmax[2] = (float)d.W; w->cmax[3] = (float)d.H;
    }
    VO_STAMP(d, 1993, 3);
}

// 32-test matcher (the reference's quirk 1, feature_matching_parallel.cpp:39-47).
// grid (match_blocks, B): frame wf = blockIdx.y of the window.  A workgroup owns 64 queries,
// lane = query (the same 64 in each of its 4 waves); the cur frame's prefixes are staged in LDS
// (16 KB at N = 4096) and wave w walks candidate quarter w with wave-uniform ds_read_b128s, four
// candidates per read, keeping two top-2 key sets per lane (even / odd candidates: independent
// chains).  The four quarters' sets merge through LDS: keys are (dist << 16 | j), so the merged
// minimum is the first-index minimum the sequential loop keeps.
__device__ __forceinline__ void top2_merge(uint32_t& m1, uint32_t& m2, uint32_t o1, uint32_t o2)
{
    const uint32_t n1v = min(m1, o1);
    m2 = min(max(m1, o1), min(m2, o2));
    m1 = n1v;
}

template <int QPL, int NW = 4>
__global__ void __launch_bounds__(64 * NW) k_match(VoDev d, int stage)
{
    constexpr int NT = 64 * NW;                      // threads; NW waves split the candidates
    const int wf = blockIdx.y;
    const VoPlan P = match_window(d, stage);
    if (wf >= vwin_records(P)) return;
    MatchFrame m;
    if (!match_header(d, stage, P, wf, m)) return;
    __shared__ unsigned s_last;
    __shared__ int s_wsum[32];
    __shared__ uint4 s_cand4[1024];                  // 4096 prefixes
    __shared__ uint2 s_top[NW - 1][QPL][64];
    uint32_t* s_cand = reinterpret_cast<uint32_t*>(s_cand4);
    const int N = d.N, n1 = m.n1, n2 = m.n2;
    // wave-uniform candidate range: scalar loop counter, key index an SGPR operand
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (blockIdx.x * (64 * QPL) < n1) {
        const uint32_t* cand = d.pre + (size_t)m.cur * N;
        for (int j0 = threadIdx.x; j0 < n2; j0 += 4 * NT) {
            uint32_t v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = j0 + u * NT < n2 ? cand[j0 + u * NT] : 0u;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (j0 + u * NT < n2) s_cand[j0 + u * NT] = v[u];
        }
        // lane's queries: blockIdx.x * (64 * QPL) + 64 u + lane
        uint32_t qv[QPL];
#pragma unroll
        for (int u = 0; u < QPL; ++u) {
            const int q = blockIdx.x * (64 * QPL) + 64 * u + lane;
            qv[u] = q < n1 ? d.pre[(size_t)m.prev * N + q] : 0u;
        }
        // the wave's share of the candidates: [j0, j1), j0 a multiple of 4
        const int qs = ((n2 + 4 * NW - 1) / (4 * NW)) * 4;
        const int j0 = min(wave * qs, n2), j1 = min(j0 + qs, n2);
        uint32_t a1[QPL], a2[QPL], b1[QPL], b2[QPL];
#pragma unroll
        for (int u = 0; u < QPL; ++u) a1[u] = a2[u] = b1[u] = b2[u] = 0xFFFFFFFFu;
        __syncthreads();
        int j = j0;
        for (; j + 4 <= j1; j += 4) {
            const uint4 c = s_cand4[j >> 2];
#pragma unroll
            for (int u = 0; u < QPL; ++u) {
                top2_insert2(((uint32_t)__popc(qv[u] ^ c.x) << 16) | (uint32_t)j,
                             ((uint32_t)__popc(qv[u] ^ c.y) << 16) | (uint32_t)(j + 1), a1[u], a2[u]);
                top2_insert2(((uint32_t)__popc(qv[u] ^ c.z) << 16) | (uint32_t)(j + 2),
                             ((uint32_t)__popc(qv[u] ^ c.w) << 16) | (uint32_t)(j + 3), b1[u], b2[u]);
            }
        }
        for (; j < j1; ++j) {
            const uint32_t cj = s_cand[j];
#pragma unroll
            for (int u = 0; u < QPL; ++u) top2_insert(((uint32_t)__popc(qv[u] ^ cj) << 16) | (uint32_t)j, a1[u], a2[u]);
        }
#pragma unroll
        for (int u = 0; u < QPL; ++u) {
            top2_merge(a1[u], a2[u], b1[u], b2[u]);
            if (wave > 0) s_top[wave - 1][u][lane] = make_uint2(a1[u], a2[u]);
        }
        __syncthreads();
        if (wave == 0) {
#pragma unroll
            for (int u = 0; u < QPL; ++u) {
#pragma unroll
                for (int w = 0; w < NW - 1; ++w) {
                    const uint2 o = s_top[w][u][lane];
                    top2_merge(a1[u], a2[u], o.x, o.y);
                }
                const int q = blockIdx.x * (64 * QPL) + 64 * u + lane;
                if (q < n1) st_sc1(m.match_j + q, ratio_accept(a1[u], a2[u], d.ratio));
            }
        }
    }
    if (blockIdx.x == 0) VO_STAMP(d, 1993, 1);
    if (!arrive_last(&m.w->ctr[0], gridDim.x, &s_last)) return;
    match_compact(d, wf, m, s_wsum);
}

// Full-length 512-test matcher (matching_serial.cpp:24-40,58; config 4's LDS descriptor-tile
// stress).  Lane = query: each thread holds its query's 512 bits in 16 VGPRs and keeps its own
// top-2 keys, so no cross-lane merge is needed.  The cur frame's descriptors stream through an
// LDS tile of MT512_TILE candidates (64 KB: 4096 x 64 B does not fit the CU's 160 KB); every
// wave walks the tile in candidate order with wave-uniform (broadcast) ds_read_b128s, so the
// top-2 update sees j ascending and the min key (dist << 16 | j) is the first-index minimum.
#define MT512_TILE 1024
// popcount-accumulate as one v_bcnt_u32_b32 (left to itself the compiler splits the chain into
// bcnt-with-0 plus v_add3: 43 instead of 35 VALU per (query, candidate) pair)
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc)
{
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}
// Hamming distance of a query (16 words) to one staged candidate (four 16-byte LDS words)
__device__ __forceinline__ uint32_t dist512(const uint32_t (&qw)[16], const uint4* c)
{
    const uint4 c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3];
    uint32_t dist = __popc(qw[0] ^ c0.x);
    dist = bcnt_acc(qw[1] ^ c0.y, dist);
    dist = bcnt_acc(qw[2] ^ c0.z, dist);
    dist = bcnt_acc(qw[3] ^ c0.w, dist);
    dist = bcnt_acc(qw[4] ^ c1.x, dist);
    dist = bcnt_acc(qw[5] ^ c1.y, dist);
    dist = bcnt_acc(qw[6] ^ c1.z, dist);
    dist = bcnt_acc(qw[7] ^ c1.w, dist);
    dist = bcnt_acc(qw[8] ^ c2.x, dist);
    dist = bcnt_acc(qw[9] ^ c2.y, dist);
    dist = bcnt_acc(qw[10] ^ c2.z, dist);
    dist = bcnt_acc(qw[11] ^ c2.w, dist);
    dist = bcnt_acc(qw[12] ^ c3.x, dist);
    dist = bcnt_acc(qw[13] ^ c3.y, dist);
    dist = bcnt_acc(qw[14] ^ c3.z, dist);
    return bcnt_acc(qw[15] ^ c3.w, dist);
}

__global__ void __launch_bounds__(256) k_match512(VoDev d, int stage)
{
    const int wf = blockIdx.y;
    const VoPlan P = match_window(d, stage);
    if (wf >= vwin_records(P)) return;
    MatchFrame m;
    if (!match_header(d, stage, P, wf, m)) return;
    __shared__ unsigned s_last;
    __shared__ int s_wsum[32];                      // match_compact: 8 rounds x 4 waves
    extern __shared__ uint4 s_tile[];        // MT512_TILE x 64 B
    const int N = d.N, n1 = m.n1, n2 = m.n2;
    const int q = blockIdx.x * MT512_QPB + threadIdx.x;
    const bool wave_live = __builtin_amdgcn_readfirstlane(blockIdx.x * MT512_QPB + (threadIdx.x & ~63)) < n1;
    if (blockIdx.x * MT512_QPB < n1) {
        uint32_t qw[16];
        {
            const uint4* qd = reinterpret_cast<const uint4*>(d.desc + ((size_t)m.prev * N + (q < n1 ? q : 0)) * 8);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const uint4 v = qd[g];
                qw[4 * g] = v.x; qw[4 * g + 1] = v.y; qw[4 * g + 2] = v.z; qw[4 * g + 3] = v.w;
            }
        }
        uint32_t m1 = 0xFFFFFFFFu, m2 = 0xFFFFFFFFu;
        const uint4* cd = reinterpret_cast<const uint4*>(d.desc + (size_t)m.cur * N * 8);
        for (int t0 = 0; t0 < n2; t0 += MT512_TILE) {
            const int nt = min(MT512_TILE, n2 - t0);
            __syncthreads();                                  // the previous tile is consumed
            for (int c = threadIdx.x; c < nt * 4; c += 256) s_tile[c] = cd[(size_t)t0 * 4 + c];
            __syncthreads();
            if (wave_live) {
                // two candidates per iteration: their LDS reads are in flight together
                int j = 0;
                for (; j + 1 < nt; j += 2) {
                    const uint32_t da = dist512(qw, s_tile + 4 * j), db = dist512(qw, s_tile + 4 * j + 4);
                    top2_insert((da << 16) | (uint32_t)(t0 + j), m1, m2);
                    top2_insert((db << 16) | (uint32_t)(t0 + j + 1), m1, m2);
                }
                if (j < nt) top2_insert((dist512(qw, s_tile + 4 * j) << 16) | (uint32_t)(t0 + j), m1, m2);
            }
        }
        if (q < n1) st_sc1(m.match_j + q, ratio_accept(m1, m2, d.ratio));
    }
    if (!arrive_last(&m.w->ctr[0], gridDim.x, &s_last)) return;
    match_compact(d, wf, m, s_wsum);
}


// ---------------------------------------------------------------------------
// RANSAC: every hypothesis k < max_hyp in one launch, one per wavefront (ransac.cpp:138-176);
// the last workgroup replays the adaptive stopping rule (ransac.cpp:139-190) over the
// per-hypothesis counts, which selects exactly the sequential loop's best hypothesis.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double shfl_d(double v, int src) { return __shfl(v, src); }
__device__ __forceinline__ double shfl_xor_d(double v, int m) { return __shfl_xor(v, m); }

// wave-wide max of a double, in every lane: DPP within rows of 16 (quad_perm 1032, 2301,
// row_half_mirror, row_mirror), then the 4 row maxima via readlane.  No LDS round trips.
__device__ __forceinline__ double dpp_f64(double v, int ctrl_sel)
{
    // every lane of every row is written by these patterns (quad_perm, row_half_mirror, row_mirror),
    // so the moves need no old value: mov_dpp lets the compiler drop the copy (and fold the move
    // into its consumer where it can)
    long long x = __double_as_longlong(v);
    int lo = (int)(x & 0xFFFFFFFFll), hi = (int)(x >> 32);
    int lo2, hi2;
    switch (ctrl_sel) {
    case 0: lo2 = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, true); hi2 = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, true); break;
    case 1: lo2 = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xF, 0xF, true); hi2 = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xF, 0xF, true); break;
    case 2: lo2 = __builtin_amdgcn_mov_dpp(lo, 0x141, 0xF, 0xF, true); hi2 = __builtin_amdgcn_mov_dpp(hi, 0x141, 0xF, 0xF, true); break;
    default: lo2 = __builtin_amdgcn_mov_dpp(lo, 0x140, 0xF, 0xF, true); hi2 = __builtin_amdgcn_mov_dpp(hi, 0x140, 0xF, 0xF, true); break;
    }
    return __longlong_as_double(((long long)hi2 << 32) | (unsigned)lo2);
}

__device__ __forceinline__ double rdlane(double v, int l);


__device__ __forceinline__ double wave_max_f64(double v)
{
    v = fmax(v, dpp_f64(v, 0));
    v = fmax(v, dpp_f64(v, 1));
    v = fmax(v, dpp_f64(v, 2));
    v = fmax(v, dpp_f64(v, 3));
    return fmax(fmax(rdlane(v, 0), rdlane(v, 16)), fmax(rdlane(v, 32), rdlane(v, 48)));
}

__device__ __forceinline__ double rdlane(double v, int l)
{
    long long x = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readlane((int)(x & 0xFFFFFFFFll), l);
    int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Sampson inlier test (computeSampsonError < thr, ransac.cpp:12-23,163-166).  For thr == 1
// the division is skipped: with den >= 1e-12, RN(num/den) < 1  <=>  num < den (exact; NaN
// and inf cases agree), tests/test_sampson_no_div.py.
__device__ __forceinline__ bool sampson_inlier(const double* F, double x, double y, double xp, double yp,
                                               double thr, bool thr_is_one)
{
    double Fx0 = (F[0] * x + F[1] * y) + F[2] * 1.0;
    double Fx1 = (F[3] * x + F[4] * y) + F[5] * 1.0;
    double Ft0 = (F[0] * xp + F[3] * yp) + F[6] * 1.0;
    double Ft1 = (F[1] * xp + F[4] * yp) + F[7] * 1.0;
    double Ft2 = (F[2] * xp + F[5] * yp) + F[8] * 1.0;
    double v = (Ft0 * x + Ft1 * y) + Ft2 * 1.0;
    double num = v * v;
    double den = ((Fx0 * Fx0 + Fx1 * Fx1) + Ft0 * Ft0) + Ft1 * Ft1;
    if (den < 1e-12) return 1.7976931348623157e308 < thr;
    return thr_is_one ? (num < den) : (num / den < thr);
}

// ---- eight hypotheses per wave: lane = 8 h + r, hypothesis h, design-matrix row r ----
// The sample, the normalisation, the 3x3 algebra (denormalize, rank 2) and the 8x9 rows are
// per lane group; one instruction serves eight hypotheses (the single-hypothesis wave spent
// most of its instructions on work that is uniform across the wave).

// DPP within 8-lane groups: lane ^ 1, lane ^ 2 (quad_perm), the other quad (row_half_mirror)
__device__ __forceinline__ int dpp_g8(int v, int step)
{
    switch (step) {
    case 0: return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);
    case 1: return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);
    default: return __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true);
    }
}
// lane q of each 8-lane group -> every lane of the group (ds_swizzle bitmask mode:
// and_mask 0x18, or_mask q)
template <int Q>
__device__ __forceinline__ int g8_bcast(int v)
{
    return __builtin_amdgcn_ds_swizzle(v, 0x18 | (Q << 5));
}
template <int Q>
__device__ __forceinline__ double g8_bcast_d(double v)
{
    const long long x = __double_as_longlong(v);
    const int lo = g8_bcast<Q>((int)(x & 0xFFFFFFFFll)), hi = g8_bcast<Q>((int)(x >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// a[c] for a group-uniform runtime column c (9-way select)
#ifndef RS_FASTSEL
#define RS_FASTSEL 1
#endif
#define RS_GROUPS_MAX 32       // lane groups of eight per workgroup (k_ransac_hyp<4>: 256 threads)
__device__ __forceinline__ double sel9(const double (&a)[9], int c)
{
#if RS_FASTSEL
    // a[c], c in [0, 8], as a select tree on the bits of c: four masks, each reused
    const bool b0 = (c & 1) != 0, b1 = (c & 2) != 0, b2 = (c & 4) != 0, b3 = (c & 8) != 0;
    const double v01 = b0 ? a[1] : a[0], v23 = b0 ? a[3] : a[2], v45 = b0 ? a[5] : a[4], v67 = b0 ? a[7] : a[6];
    const double v03 = b1 ? v23 : v01, v47 = b1 ? v67 : v45;
    const double v07 = b2 ? v47 : v03;
    return b3 ? a[8] : v07;
#else
    double v = a[0];
#pragma unroll
    for (int j = 1; j < 9; ++j) v = c == j ? a[j] : v;
    return v;
#endif
}

#ifndef RS_FASTRED
#define RS_FASTRED 1                   // Gauss-Jordan pivot: group max, then min index among the maxima
#endif
#ifndef RS_LDSPIV
#define RS_LDSPIV 1                    // Gauss-Jordan pivot row through LDS (else lane shuffles)
#endif
#define RS_ROWSTRIDE 10                // doubles per lane row in LDS (16-byte aligned rows)
// computeFundamentalMatrix on a minimal sample (ransac.cpp:63-93) for the lane group's
// hypothesis: Gauss-Jordan with complete pivoting exactly as oracle nullvec_8x9 (pivot = max
// |a| over unused rows/cols, ties to the first in row-major order), lane r holding row r.
__device__ void fit_F8_group(const double* __restrict__ pts, const int s8[8], int r, int gbase, double F[9],
                             [[maybe_unused]] const VoDev* sd = nullptr, [[maybe_unused]] int sk = 0)
{
    double P[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double2* p = reinterpret_cast<const double2*>(pts + 4 * (size_t)s8[i]);
        double2 a = p[0], b = p[1];
        P[i][0] = a.x; P[i][1] = a.y; P[i][2] = b.x; P[i][3] = b.y;
    }
    double mx1 = 0, my1 = 0, mx2 = 0, my2 = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) { mx1 = mx1 + P[i][0]; my1 = my1 + P[i][1]; mx2 = mx2 + P[i][2]; my2 = my2 + P[i][3]; }
    mx1 = mx1 / 8.0; my1 = my1 / 8.0; mx2 = mx2 / 8.0; my2 = my2 / 8.0;
    double sc1 = 0, sc2 = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        double a = P[i][0] - mx1, b = P[i][1] - my1, c = P[i][2] - mx2, e = P[i][3] - my2;
        sc1 = sc1 + (a * a + b * b);
        sc2 = sc2 + (c * c + e * e);
    }
    sc1 = sqrt(2.0) / sqrt(sc1 / 8.0);
    sc2 = sqrt(2.0) / sqrt(sc2 / 8.0);
#ifdef VO_STAMPS
    if (sd) { __builtin_amdgcn_s_waitcnt(0); VO_STAMP(*sd, sk, 3); }   // points loaded, normalisation done
#endif
    const double o1x = -(sc1 * mx1), o1y = -(sc1 * my1), o2x = -(sc2 * mx2), o2y = -(sc2 * my2);
    double x1 = 0, y1 = 0, x2 = 0, y2 = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (i == r) { x1 = P[i][0]; y1 = P[i][1]; x2 = P[i][2]; y2 = P[i][3]; }
    double a[9];
    design_row(sc1 * x1 + o1x, sc1 * y1 + o1y, sc2 * x2 + o2x, sc2 * y2 + o2y, a);
    uint32_t used_c = 0, used_r = 0;
    int my_pc = -1;                                 // the column this row pivoted (if it did)
    bool live = true;                               // the group's elimination still runs
#pragma unroll
    for (int step = 0; step < 8; ++step) {
        // lane-local candidate: first max |a| over the unused columns of an unused row
        double bv = -1.0;
        int bi = 1 << 30;
#if RS_FASTSEL
        // the same first maximum as a tournament (depth 4 instead of a 9-step compare / select
        // chain): candidates are |a| over unused columns, > 0, else -1; a later one wins only if
        // strictly greater, so ties go to the smaller column
        {
            double mv[9];
#pragma unroll
            for (int c = 0; c < 9; ++c) {
                const double v = fabs(a[c]);
                mv[c] = (!((used_c >> c) & 1u) && v > 0.0) ? v : -1.0;
            }
            auto win = [](double& va, int& ia, double vb, int ib) {
                const bool t = vb > va;
                va = t ? vb : va;
                ia = t ? ib : ia;
            };
            double w0 = mv[0], w1 = mv[2], w2 = mv[4], w3 = mv[6];
            int i0 = 0, i1 = 2, i2 = 4, i3 = 6;
            win(w0, i0, mv[1], 1); win(w1, i1, mv[3], 3); win(w2, i2, mv[5], 5); win(w3, i3, mv[7], 7);
            win(w0, i0, w1, i1); win(w2, i2, w3, i3);
            win(w0, i0, w2, i2);
            win(w0, i0, mv[8], 8);
            if (!((used_r >> r) & 1u) && w0 > 0.0) { bv = w0; bi = r * 16 + i0; }
        }
#else
        if (!((used_r >> r) & 1u)) {
#pragma unroll
            for (int c = 0; c < 9; ++c) {
                const double v = fabs(a[c]);
                if (!((used_c >> c) & 1u) && v > 0.0 && v > bv) { bv = v; bi = r * 16 + c; }
            }
        }
#endif
        // group maximum, ties to the smaller flat index: the maximum value first (three DPP max
        // steps; candidates are positive or -1, never NaN), then the smallest index among the lanes
        // holding it (three DPP min steps) -- the same pivot as the pairwise (value, index) reduction
        // with its compare / select chains
#if RS_FASTRED
        {
            double gm = bv;
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const double o = dpp_f64(gm, t);
                asm volatile("v_max_f64 %0, %1, %2" : "=v"(gm) : "v"(gm), "v"(o));   // no NaN: no canonicalising max
            }
            int ci = bv == gm ? bi : (1 << 30);
#pragma unroll
            for (int t = 0; t < 3; ++t) ci = min(ci, dpp_g8(ci, t));
            bv = gm;
            bi = ci;
        }
#else
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const double ov = dpp_f64(bv, t);
            const int oi = dpp_g8(bi, t);
            const bool take = ov > bv || (ov == bv && oi < bi);
            bv = take ? ov : bv;
            bi = take ? oi : bi;
        }
#endif
        live = live && bv > 0.0;                    // rank deficient: remaining columns free
        // (flat index r * 16 + c: the same order as r * 9 + c, row and column by shift and mask)
        const int pr = bi >> 4, pc = bi & 15;
#if RS_LDSPIV
        // the pivot row, A[r][pc] and the pivot through LDS: each lane stores its row, then reads
        // the group's pivot row and its own entry in column pc (12 LDS instructions instead of 20
        // lane shuffles and a nine-way select).  One wave's lanes only, ordered by wave barriers.
        double prow[9], arpc, piv;
        {
            __shared__ __attribute__((aligned(16))) double s_row[RS_GROUPS_MAX * 8][RS_ROWSTRIDE];
            double* mine = s_row[threadIdx.x];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();              // the previous step's reads are done
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int c = 0; c < 8; c += 2) *reinterpret_cast<double2*>(mine + c) = make_double2(a[c], a[c + 1]);
            mine[8] = a[8];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const double* prw = s_row[(threadIdx.x & ~7u) + (live ? pr : 0)];
#pragma unroll
            for (int c = 0; c < 8; c += 2) {
                const double2 v2 = *reinterpret_cast<const double2*>(prw + c);
                prow[c] = v2.x; prow[c + 1] = v2.y;
            }
            prow[8] = prw[8];
            const int pcc = live ? pc : 0;
            arpc = mine[pcc];
            piv = prw[pcc];
        }
#else
        const double arpc = sel9(a, live ? pc : 0);   // A[r][pc]
        const int src = gbase + (live ? pr : 0);
        const double piv = __shfl(arpc, src);
        double prow[9];
#pragma unroll
        for (int c = 0; c < 9; ++c) prow[c] = __shfl(a[c], src);
#endif
        if (live) {
            used_r |= 1u << pr; used_c |= 1u << pc;
            if (r == pr) my_pc = pc;
            if (r != pr) {
                const double fct = arpc / piv;
#pragma unroll
                for (int c = 0; c < 9; ++c) a[c] = a[c] - fct * prow[c];
            }
        }
    }
#ifdef VO_STAMPS
    if (sd) VO_STAMP(*sd, sk, 4);                   // Gauss-Jordan done
#endif
    int fc = 0;
#pragma unroll
    for (int j = 8; j >= 0; --j) if (!((used_c >> j) & 1u)) fc = j;
    // back substitution: x_fc = 1, x_pc = -a[pr][fc] / a[pr][pc] from each pivot row
    const double val = my_pc >= 0 ? -(sel9(a, fc) / sel9(a, my_pc)) : 0.0;
    double f[9];
#if RS_FASTSEL
    // the group's solution vector through LDS: each pivot row stores its x_pc at column pc, the
    // free column holds 1, the rest 0 -- the same vector as eight broadcast rows selected into
    // nine registers (72 compare / select pairs, each padded for its VCC read), in three LDS
    // steps.  One wave's lanes only, ordered by wave barriers.
    {
        __shared__ double s_fb[RS_GROUPS_MAX][9];
        double* fb = s_fb[threadIdx.x >> 3];
        fb[r] = 0.0;
        if (r == 0) fb[8] = 0.0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (my_pc >= 0) fb[my_pc] = val;
        if (r == 0) fb[fc] = 1.0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int j = 0; j < 9; ++j) f[j] = fb[j];
        __builtin_amdgcn_wave_barrier();              // the next hypothesis' fit rewrites fb
    }
#else
#pragma unroll
    for (int j = 0; j < 9; ++j) f[j] = (j == fc) ? 1.0 : 0.0;
    auto take_row = [&](int cq, double vq) {
#pragma unroll
        for (int j = 0; j < 9; ++j) f[j] = cq == j ? vq : f[j];
    };
    take_row(g8_bcast<0>(my_pc), g8_bcast_d<0>(val));
    take_row(g8_bcast<1>(my_pc), g8_bcast_d<1>(val));
    take_row(g8_bcast<2>(my_pc), g8_bcast_d<2>(val));
    take_row(g8_bcast<3>(my_pc), g8_bcast_d<3>(val));
    take_row(g8_bcast<4>(my_pc), g8_bcast_d<4>(val));
    take_row(g8_bcast<5>(my_pc), g8_bcast_d<5>(val));
    take_row(g8_bcast<6>(my_pc), g8_bcast_d<6>(val));
    take_row(g8_bcast<7>(my_pc), g8_bcast_d<7>(val));
#endif
    double nn = 0.0;
#pragma unroll
    for (int j = 0; j < 9; ++j) nn = nn + f[j] * f[j];
    nn = sqrt(nn);
#pragma unroll
    for (int j = 0; j < 9; ++j) f[j] = f[j] / nn;
    denormalize(f, sc1, mx1, my1, sc2, mx2, my2, F);   // (rank 2 by the caller: rank2(F))
}

// inliers of the group's F among the first `scored` matches: lane r tests matches 8 j + r of
// each 64-match word, the group's byte of each ballot is shifted into the word (bit i = match
// i); the words go to `mask` (k_refit compacts the best set from it)
// Two forms by register budget: the batched launches (k_ransac_hyp: many waves per SIMD) take four
// chains and no prefetch (152 VGPRs, 3 waves per SIMD); the latency launches (k_ransac_fused: the
// per-frame call and the stage API, about one wave per SIMD) take eight chains and the prefetch.
#ifndef RS_HYP_J
#define RS_HYP_J 4                     // Sampson chains in flight per lane
#endif
#ifndef RS_HYP_PF
#define RS_HYP_PF 0                    // the next word's points loaded before this word's tests
#endif
#ifndef RS_EARLY
#define RS_EARLY 1                     // later chunks: a wave's count stops once it cannot pass the best
#endif
#ifndef RS_FUSED_J
#define RS_FUSED_J 8
#endif
#ifndef RS_FUSED_PF
#define RS_FUSED_PF 1
#endif
// The word's eight Sampson tests as one branch-free stream (each step over j = 0..7, so eight
// independent f64 chains are in flight), the threshold form hoisted out of the loop, and the next
// word's points loaded before this word's tests.  The per-match arithmetic is sampson_inlier's,
// operation for operation (computeSampsonError, ransac.cpp:12-23): the same values, the same
// roundings.  (The single-chain form it replaced issued one Sampson at a time behind two exec-mask
// branches: 4.3k cycles per word for a lone wave.)  w0, ws: the words w0, w0 + ws, ... (a split count)
// bound >= 0 (a later chunk of the pose pass): the count stops once no hypothesis of the wave can
// end above `bound`, the previous replay's best -- the sequential loop only takes a count above its
// running best, which is at least that.  Such a count is left partial (still <= bound, so the
// replay decides the same) and so are its mask words (k_refit reads only the best hypothesis').
template <bool ONE, int RS_COUNT_J, bool RS_COUNT_PREFETCH>
__device__ __forceinline__ int count_words(const double* __restrict__ pts, int scored, const double* F, double thr,
                                           int h, int r, bool store, uint64_t* __restrict__ mask, int bound,
                                           int w0 = 0, int ws = 1)
{
    const int nw = (scored + 63) >> 6;
    const bool deg_in = 1.7976931348623157e308 < thr;     // sampson() of a degenerate match
    const double F0 = F[0], F1 = F[1], F2 = F[2], F3 = F[3], F4 = F[4], F5 = F[5], F6 = F[6], F7 = F[7], F8 = F[8];
    int cnt = 0;
    double2 a[8], c[8];
    auto ld = [&](int w) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int i = min(w * 64 + j * 8 + r, scored - 1);   // in range; lanes past scored test nothing
            const double2* p = reinterpret_cast<const double2*>(pts + 4 * (size_t)i);
            a[j] = p[0]; c[j] = p[1];
        }
    };
    if (RS_COUNT_PREFETCH && w0 < nw) ld(w0);
    for (int w = w0; w < nw; w += ws) {
        if (!RS_COUNT_PREFETCH) ld(w);
        double x[8], y[8], xp[8], yp[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { x[j] = a[j].x; y[j] = a[j].y; xp[j] = c[j].x; yp[j] = c[j].y; }
        if (RS_COUNT_PREFETCH && w + ws < nw) ld(w + ws);
        // the word's bits as lane masks (each test one v_cmp into SGPRs, combined by the scalar
        // unit), then the group's byte of each mask into byte j of the lane's word: a per-lane
        // 64-bit shift and one v_perm_b32 per j
        uint32_t wlo = 0u, whi = 0u;
        const unsigned sh = 8u * (unsigned)h;
#pragma unroll
        for (int q = 0; q < 8; q += RS_COUNT_J) {          // RS_COUNT_J chains in flight
            double Fx0[RS_COUNT_J], Fx1[RS_COUNT_J], Ft0[RS_COUNT_J], Ft1[RS_COUNT_J], Ft2[RS_COUNT_J], v[RS_COUNT_J];
#pragma unroll
            for (int u = 0; u < RS_COUNT_J; ++u) Fx0[u] = (F0 * x[q + u] + F1 * y[q + u]) + F2 * 1.0;
#pragma unroll
            for (int u = 0; u < RS_COUNT_J; ++u) Fx1[u] = (F3 * x[q + u] + F4 * y[q + u]) + F5 * 1.0;
#pragma unroll
            for (int u = 0; u < RS_COUNT_J; ++u) Ft0[u] = (F0 * xp[q + u] + F3 * yp[q + u]) + F6 * 1.0;
#pragma unroll
            for (int u = 0; u < RS_COUNT_J; ++u) Ft1[u] = (F1 * xp[q + u] + F4 * yp[q + u]) + F7 * 1.0;
#pragma unroll
            for (int u = 0; u < RS_COUNT_J; ++u) Ft2[u] = (F2 * xp[q + u] + F5 * yp[q + u]) + F8 * 1.0;
#pragma unroll
            for (int u = 0; u < RS_COUNT_J; ++u) v[u] = (Ft0[u] * x[q + u] + Ft1[u] * y[q + u]) + Ft2[u] * 1.0;
#pragma unroll
            for (int u = 0; u < RS_COUNT_J; ++u) {
                const int j = q + u;
                const double num = v[u] * v[u];
                const double den = ((Fx0[u] * Fx0[u] + Fx1[u] * Fx1[u]) + Ft0[u] * Ft0[u]) + Ft1[u] * Ft1[u];
                const unsigned long long dg = ballot64(den < 1e-12);          // sampson() = DBL_MAX
                unsigned long long bal;
                if constexpr (ONE) bal = ballot64(num < den) & ~dg;      // num / den < 1.0 exactly when num < den
                else bal = (ballot64(num / den < thr) & ~dg) | (deg_in ? dg : 0ull);
                bal &= ballot64(w * 64 + j * 8 + r < scored);
                const uint32_t b = (uint32_t)(bal >> sh);                    // byte 0: this group's tests
                // byte j of the half-word from b's byte 0, the other bytes kept (selector 4 + k: byte k of
                // the first operand; 0: byte 0 of the second)
                constexpr uint32_t keep = 0x07060504u;
                const uint32_t sel = keep & ~(0xFFu << (8 * (j & 3)));
                if (j < 4) wlo = __builtin_amdgcn_perm(wlo, b, sel);
                else whi = __builtin_amdgcn_perm(whi, b, sel);
            }
        }
        const uint64_t word = (uint64_t)wlo | ((uint64_t)whi << 32);
        cnt += __popcll(word);
        if (store && r == (w & 7)) mask[w] = word;
        if (bound >= 0 && ballot64(store && cnt + max(scored - (w + 1) * 64, 0) > bound) == 0ull) break;
    }
    return cnt;
}
// One hypothesis per wave (the latency form): lane L tests match 64 w + L, four words in flight, and
// the ballot is the mask word itself.  The same per-match arithmetic as count_words.
template <bool ONE>
__device__ __forceinline__ int count_wave(const double* __restrict__ pts, int scored, const double* F, double thr,
                                          int lane, bool store, uint64_t* __restrict__ mask, int bound)
{
    const int nw = (scored + 63) >> 6;
    const bool deg_in = 1.7976931348623157e308 < thr;
    const double F0 = F[0], F1 = F[1], F2 = F[2], F3 = F[3], F4 = F[4], F5 = F[5], F6 = F[6], F7 = F[7], F8 = F[8];
    int cnt = 0;
    for (int w0 = 0; w0 < nw; w0 += 4) {
        double x[4], y[4], xp[4], yp[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = min((w0 + u) * 64 + lane, scored - 1);
            const double2* p = reinterpret_cast<const double2*>(pts + 4 * (size_t)i);
            const double2 a = p[0], c = p[1];
            x[u] = a.x; y[u] = a.y; xp[u] = c.x; yp[u] = c.y;
        }
        double Fx0[4], Fx1[4], Ft0[4], Ft1[4], Ft2[4], v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) Fx0[u] = (F0 * x[u] + F1 * y[u]) + F2 * 1.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) Fx1[u] = (F3 * x[u] + F4 * y[u]) + F5 * 1.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) Ft0[u] = (F0 * xp[u] + F3 * yp[u]) + F6 * 1.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) Ft1[u] = (F1 * xp[u] + F4 * yp[u]) + F7 * 1.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) Ft2[u] = (F2 * xp[u] + F5 * yp[u]) + F8 * 1.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = (Ft0[u] * x[u] + Ft1[u] * y[u]) + Ft2[u] * 1.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int w = w0 + u;
            if (w < nw) {                                  // wave-uniform
                const double num = v[u] * v[u];
                const double den = ((Fx0[u] * Fx0[u] + Fx1[u] * Fx1[u]) + Ft0[u] * Ft0[u]) + Ft1[u] * Ft1[u];
                const unsigned long long dg = ballot64(den < 1e-12);
                unsigned long long bal;
                if constexpr (ONE) bal = ballot64(num < den) & ~dg;
                else bal = (ballot64(num / den < thr) & ~dg) | (deg_in ? dg : 0ull);
                bal &= ballot64(w * 64 + lane < scored);
                cnt += __popcll(bal);
                if (store && lane == 0) mask[w] = bal;
            }
        }
        if (bound >= 0 && !(store && cnt + max(scored - (w0 + 4) * 64, 0) > bound)) break;   // wave-uniform
    }
    return cnt;
}
// The same count through the f32 certificate (vo_sampson32.h; thr == 1): each match's decision is
// taken in f32 where the error bound proves it equal to the f64 test's, two matches per packed
// instruction, and by sampson_inlier's f64 arithmetic for the rest (a word's undecided matches,
// wave-uniform branch; a hypothesis whose constants are not finite sends all its matches there).
// Lane r reads components of its matches 64 w + 8 j + r from the word-swizzled pts32 block as
// float4s (j = 4 q .. 4 q + 3), so a packed pair is a register pair as loaded.  The word's bits, the
// mask store and the early stop are count_words'.
typedef float vo_f2 __attribute__((ext_vector_type(2)));
#ifndef RS_S32
#define RS_S32 1                       // 0: the f64 count for every match (the certificate off)
#endif
__device__ __forceinline__ int count_words32(const double* __restrict__ pts, const float* __restrict__ pts32, int scored,
                                             const double* F, const float* cmax, int h, int r, bool store,
                                             uint64_t* __restrict__ mask, int bound, int w0, int ws)
{
    const int nw = (scored + 63) >> 6;
    VoS32 s;
    vo_s32_setup(F, cmax, &s);
    const auto fma2 = [](vo_f2 a, vo_f2 b, vo_f2 c) { return __builtin_elementwise_fma(a, b, c); };
    const auto abs2 = [](vo_f2 a) { return __builtin_elementwise_abs(a); };
    int cnt = 0;
    for (int w = w0; w < nw; w += ws) {
        float4 L[4][2];                                // [component][q]: matches j = 4 q .. 4 q + 3
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int q = 0; q < 2; ++q)
                L[c][q] = *reinterpret_cast<const float4*>(pts32 + (size_t)w * 256 + c * 64 + q * 32 + r * 4);
        int dec[8];
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int e = 0; e < 2; ++e) {              // the pair j = 4 q + 2 e, + 1
                const vo_f2 x = e ? vo_f2{L[0][q].z, L[0][q].w} : vo_f2{L[0][q].x, L[0][q].y};
                const vo_f2 y = e ? vo_f2{L[1][q].z, L[1][q].w} : vo_f2{L[1][q].x, L[1][q].y};
                const vo_f2 xp = e ? vo_f2{L[2][q].z, L[2][q].w} : vo_f2{L[2][q].x, L[2][q].y};
                const vo_f2 yp = e ? vo_f2{L[3][q].z, L[3][q].w} : vo_f2{L[3][q].x, L[3][q].y};
                vo_f2 diff, bnd, den;
                vo_s32_eval(s, x, y, xp, yp, fma2, abs2, &diff, &bnd, &den);
                dec[4 * q + 2 * e] = vo_s32_decide(diff.x, bnd.x, den.x);
                dec[4 * q + 2 * e + 1] = vo_s32_decide(diff.y, bnd.y, den.y);
            }
        bool und = false;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const bool valid = w * 64 + j * 8 + r < scored;
            if (!s.ok || !RS_S32) dec[j] = -1;
            und |= valid && dec[j] < 0;
        }
        if (ballot64(und) != 0ull) {                   // wave-uniform: the f64 test where f32 cannot decide
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int i = w * 64 + j * 8 + r;
                if (dec[j] < 0 && i < scored) {
                    const double2* p = reinterpret_cast<const double2*>(pts + 4 * (size_t)i);
                    const double2 a = p[0], c = p[1];
                    dec[j] = sampson_inlier(F, a.x, a.y, c.x, c.y, 1.0, true) ? 1 : 0;
                }
            }
        }
        uint32_t wlo = 0u, whi = 0u;
        const unsigned sh = 8u * (unsigned)h;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const unsigned long long bal = ballot64(dec[j] == 1 && w * 64 + j * 8 + r < scored);
            const uint32_t b = (uint32_t)(bal >> sh);
            constexpr uint32_t keep = 0x07060504u;
            const uint32_t sel = keep & ~(0xFFu << (8 * (j & 3)));
            if (j < 4) wlo = __builtin_amdgcn_perm(wlo, b, sel);
            else whi = __builtin_amdgcn_perm(whi, b, sel);
        }
        const uint64_t word = (uint64_t)wlo | ((uint64_t)whi << 32);
        cnt += __popcll(word);
        if (store && r == (w & 7)) mask[w] = word;
        if (bound >= 0 && ballot64(store && cnt + max(scored - (w + 1) * 64, 0) > bound) == 0ull) break;
    }
    return cnt;
}
// count_wave through the f32 certificate (thr == 1): lane L tests match 64 w + L of four words in
// flight, each an f32 chain (scalar: the latency form), the f64 test where f32 cannot decide
__device__ __forceinline__ int count_wave32(const double* __restrict__ pts, const float* __restrict__ pts32, int scored,
                                            const double* F, const float* cmax, int lane, bool store,
                                            uint64_t* __restrict__ mask, int bound)
{
    const int nw = (scored + 63) >> 6;
    VoS32 s;
    vo_s32_setup(F, cmax, &s);
    const auto fma1 = [](float a, float b, float c) { return __builtin_fmaf(a, b, c); };
    const auto abs1 = [](float a) { return __builtin_fabsf(a); };
    const int j = lane >> 3, r = lane & 7;
    const int lo = (j >> 2) * 32 + r * 4 + (j & 3);           // vo_pts32_index of match 64 w + lane, less 256 w
    int cnt = 0;
    for (int w0 = 0; w0 < nw; w0 += 4) {
        int dec[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float* q = pts32 + (size_t)min(w0 + u, nw - 1) * 256 + lo;
            float diff, bnd, den;
            vo_s32_eval(s, q[0], q[64], q[128], q[192], fma1, abs1, &diff, &bnd, &den);
            dec[u] = (s.ok && RS_S32) ? vo_s32_decide(diff, bnd, den) : -1;
        }
        bool und = false;
#pragma unroll
        for (int u = 0; u < 4; ++u) und |= (w0 + u) * 64 + lane < scored && dec[u] < 0;
        if (ballot64(und) != 0ull) {                   // wave-uniform
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = (w0 + u) * 64 + lane;
                if (dec[u] < 0 && i < scored) {
                    const double2* p = reinterpret_cast<const double2*>(pts + 4 * (size_t)i);
                    const double2 a = p[0], c = p[1];
                    dec[u] = sampson_inlier(F, a.x, a.y, c.x, c.y, 1.0, true) ? 1 : 0;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int w = w0 + u;
            if (w < nw) {                                  // wave-uniform
                const unsigned long long bal = ballot64(dec[u] == 1 && w * 64 + lane < scored);
                cnt += __popcll(bal);
                if (store && lane == 0) mask[w] = bal;
            }
        }
        if (bound >= 0 && !(store && cnt + max(scored - (w0 + 4) * 64, 0) > bound)) break;   // wave-uniform
    }
    return cnt;
}
template <int J, bool PF>
__device__ __forceinline__ int count_inliers_group(const double* __restrict__ pts, const float* __restrict__ pts32,
                                                   const float* cmax, int scored, const double* F, double thr,
                                                   int h, int r, bool store, uint64_t* __restrict__ mask,
                                                   int bound = -1, int w0 = 0, int ws = 1)
{
    if (thr == 1.0) return count_words32(pts, pts32, scored, F, cmax, h, r, store, mask, bound, w0, ws);
    return count_words<false, J, PF>(pts, scored, F, thr, h, r, store, mask, bound, w0, ws);
}

// SVD of a 3x3 A (mirror of oracle svd3): min_eigvec3 + one 2x2 Jacobi rotation
__device__ void svd3(const double* A, double* U, double* S, double* Vt)
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
#pragma unroll
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
#pragma unroll
    for (int i = 0; i < 3; ++i) { w1[i] = c * p[i] - s * q[i]; w2[i] = s * p[i] + c * q[i]; }
    double V[9];                               /* columns: descending eigenvalue, then v3 */
    const double* va = l2 > l1 ? w2 : w1;
    const double* vb = l2 > l1 ? w1 : w2;
#pragma unroll
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


// 4x4 helpers for the GT scale (mirror of oracle inv4 / mm4)
__device__ void mm4(const double* A, const double* B, double* C)
{
    double T[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            T[i * 4 + j] = ((A[i * 4 + 0] * B[0 * 4 + j] + A[i * 4 + 1] * B[1 * 4 + j]) + A[i * 4 + 2] * B[2 * 4 + j]) +
                           A[i * 4 + 3] * B[3 * 4 + j];
    for (int i = 0; i < 16; ++i) C[i] = T[i];
}
__device__ void inv4(const double* M, double* Inv)
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

// HPB hypotheses per workgroup, WPH waves per hypothesis.  First chunk: one hypothesis per
// 4-wave workgroup (each wave fits the same F, the four split the Sampson count: the latency
// path); second chunk: four single-wave hypotheses per workgroup, since it usually exits at
// once (fewer workgroups to dispatch).
// HPB waves per workgroup, eight hypotheses per wave (lane 8 h + r: hypothesis h, row r).
// reps: hypothesis blocks per workgroup (strided by the grid), so a later chunk, which usually
// exits at once, dispatches reps times fewer workgroups
// One chunk [k0, k1) of the hypotheses on workgroups bx of nbx.  ready (the fused form): the chunk's
// replay publishes w->ready1 when it is done (k0 == 0), or the chunk waits for it first (k0 > 0).
// W1: one hypothesis per wave (the latency form: every lane group fits the same hypothesis, the
// wave's 64 lanes split its count) instead of eight
template <int HPB, int CJ, bool CPF, bool W1 = false>
__device__ __forceinline__ void ransac_chunk(const VoDev& d, int k0, int k1, int nhyp, int stage, int reps, int bx,
                                             int nbx, bool ready)
{
    constexpr int HPW = W1 ? 1 : 8;                // hypotheses per wave
    const int wf = blockIdx.y;                     // window frame
    if (wf >= vwin_count(d, stage)) return;
    VoWork* w = d.work + wf;
    if (w->status != VO_STATUS_OK) return;
    if (ready && k0 > 0) {
        // the fused launch: wait for the first chunk's replay (bounded; its four workgroups and these
        // run together -- the launch is one frame's 64 workgroups on an otherwise idle queue)
        __shared__ unsigned s_to;
        if (threadIdx.x == 0) {
            unsigned it = 0u;
            // relaxed polls, one acquire fence after the barrier (an acquire poll invalidates the
            // XCD's L2 on every iteration, under the first chunk's waves: 31.7 us vs 2 x 5.5 us)
            while (__hip_atomic_load((gu32*)&w->ready1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u &&
                   it < d.spin_limit) {
                __builtin_amdgcn_s_sleep(2);
                ++it;
            }
            s_to = it >= d.spin_limit ? 1u : 0u;
        }
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (s_to) {
            // loud, never a hang: the chunk's arrival count stays short, so no replay runs over
            // counts nobody wrote; every row from here carries err (k_finalize reads the counter) and
            // the call returns VO_ERR_INTERNAL.  The record's counters are reset by the next header
            if (threadIdx.x == 0) atomicAdd(d.ctr + VO_CTR_ERR, 1u);
            return;
        }
    }
    if (k0 > 0 && !w->need_more) return;           // the replay of [0, k0) already stopped
    __shared__ unsigned s_last;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 3, r = lane & 7;
    const int M = w->M, scored = w->scored;
    const double* pts = d.pts + (size_t)wf * 4 * d.N;
    int32_t* counts = d.counts + (size_t)wf * d.max_hyp;
    int k = k0 + (bx * HPB + wave) * HPW + (W1 ? 0 : h);
    // Hypotheses at or past the previous replay's bound are never evaluated by the sequential
    // loop: once an improvement updated maxIterations (best > 0 and its table entry is not the
    // 'denom == 0: no update' mark) and the loop went on past k0 (maxit > 100), the inlier ratio
    // is in the band where maxIterations only falls as best rises (below it the x86 INT_MIN clamp
    // gives 100, quirk 8), so maxit bounds every later hypothesis.  Otherwise maxit is still the
    // initial 1176 and the next improvement may raise it to 2000.  Hypotheses past the bound are
    // marked -1 and cost nothing.
    int kbound = k1;
    if (k0 > 0 && w->best > 0 && d.maxit_tab[(size_t)M * (M + 1) / 2 + w->best] != 0xFFFFu)
        kbound = min(w->maxit, k1);
    // counts past the previous replay's best only matter to the loop: a later chunk stops a wave's
    // count once none of its hypotheses can pass it (not the stage API, which returns every count)
    const int cbound = (RS_EARLY && k0 > 0 && !stage) ? w->best : -1;
    for (int rep = 0; rep < reps; ++rep, k += nbx * HPB * HPW) {
        const int kb = W1 ? k : k - h;             // the wave's first hypothesis
        if (kb >= k1) break;                       // wave-uniform
        const bool mine = k < kbound;
        if (__builtin_amdgcn_readfirstlane(kb) < kbound) {   // some group of the wave has work
            VO_STAMP(d, k, 0);
            int s8[8];
            if (d.rng_mode == VO_RNG_MT19937) {
                // the reference's std::sample draws, drawn on the host for this record (vo_api.cpp)
                const int4* sp = reinterpret_cast<const int4*>(d.samples + ((size_t)wf * d.max_hyp + min(k, nhyp - 1)) * 8);
                const int4 lo = sp[0], hi = sp[1];
                s8[0] = lo.x; s8[1] = lo.y; s8[2] = lo.z; s8[3] = lo.w;
                s8[4] = hi.x; s8[5] = hi.y; s8[6] = hi.z; s8[7] = hi.w;
            } else {
                sample8(w->frame_seed, min(k, nhyp - 1), M, s8);
            }
            VO_STAMP(d, k, 1);
            double F[9];
            fit_F8_group(pts, s8, r, lane & ~7, F, &d, k);
#if RS_PROBE == 1
            {   // timing probe: the fit twice (the second result only kept alive)
                double F2[9];
                fit_F8_group(pts, s8, r, lane & ~7, F2);
#pragma unroll
                for (int j = 0; j < 9; ++j) asm volatile("" ::"v"(F2[j]));
            }
#endif
            VO_STAMP(d, k, 2);
#if RS_PROBE == 2
            {   // timing probe: rank 2 twice
                double F2[9];
#pragma unroll
                for (int j = 0; j < 9; ++j) { F2[j] = F[j]; asm volatile("" : "+v"(F2[j])); }
                rank2(F2);
#pragma unroll
                for (int j = 0; j < 9; ++j) asm volatile("" ::"v"(F2[j]));
            }
#endif
            rank2(F);
            VO_STAMP(d, k, 5);
            if (mine && (!W1 || h == 0)) {
                double* hf = d.hypF + ((size_t)wf * d.max_hyp + k) * 9;
#pragma unroll
                for (int j = 0; j < 9; ++j)
                    if (j == r || (j == 8 && r == 0)) hf[j] = F[j];   // lane r: F[r]; lane 0 also F[8]
            }
            uint64_t* msk = d.inlmask + ((size_t)wf * d.max_hyp + min(k, nhyp - 1)) * d.mask_words;
            int cnt;
            if constexpr (W1)
                cnt = d.sampson_thr == 1.0 ? count_wave32(pts, d.pts32 + (size_t)wf * VO_PTS32_PER(d.N), scored, F, w->cmax,
                                                          lane, mine, msk, cbound)
                                           : count_wave<false>(pts, scored, F, d.sampson_thr, lane, mine, msk, cbound);
            else
                cnt = count_inliers_group<CJ, CPF>(pts, d.pts32 + (size_t)wf * VO_PTS32_PER(d.N), w->cmax, scored, F,
                                                   d.sampson_thr, h, r, mine, msk, cbound);
            if (mine && (W1 ? lane == 0 : r == 0)) st_sc1(counts + k, cnt);
            VO_STAMP(d, k, 6);
        }
        if (!mine && k < k1 && (W1 ? lane == 0 : r == 0)) st_sc1(counts + k, -1);   // skipped: the replay never takes it
    }
    unsigned* ctr = &w->ctr[k0 == 0 ? 1 : (k0 < VO_HYP_CHUNK1 ? 2 : 3)];   // one arrival counter per chunk
    if (!arrive_last(ctr, nbx, &s_last)) return;
    if (threadIdx.x >= 64) return;                 // the replay is one wave's
    VO_STAMP(d, 1997 + (k0 > 0), 0);
    // ---- last workgroup (one wave): replay of ransac.cpp:139-190 over [kk, k1) ----
    // 64 hypotheses at a time: their counts and adaptive-table entries are loaded once, then
    // every improvement inside the window is a ballot + two shuffles (no memory round trip)
    const uint16_t* tab = d.maxit_tab + (size_t)M * (M + 1) / 2;
    int kk, maxit, best, bestk;
    if (k0 == 0) { kk = 0; maxit = d.maxit_initial; best = 0; bestk = -1; }
    else { kk = w->k_done; maxit = w->maxit; best = w->best; bestk = w->bestk; }
    if (maxit > nhyp) maxit = nhyp;
    const int lim = k1;
    while (kk < maxit && kk < lim) {
        const int base = kk, idx = base + lane;
        const int c = idx < lim ? ld_sc1(counts + idx) : -1;
        const int u = (c >= 0 && c <= M) ? (int)tab[c] : 0xFFFF;
        for (;;) {
            const unsigned long long bal = ballot64(idx >= kk && idx < maxit && idx < lim && c > best);
            if (bal == 0ull) {
                kk = min(min(base + 64, maxit), lim);
                break;
            }
            const int j = __ffsll((long long)bal) - 1;
            best = __shfl(c, j);
            bestk = base + j;
            const int uj = __shfl(u, j);
            if (uj != 0xFFFF) maxit = min(uj, nhyp);
            kk = bestk + 1;
            if (!(kk < maxit && kk < lim)) break;
        }
    }
    VO_STAMP(d, 1997 + (k0 > 0), 1);
    if (lane == 0) {
        w->k_done = kk; w->maxit = maxit; w->best = best; w->bestk = bestk;
        w->need_more = kk < maxit ? 1 : 0;
        w->n_eval = kk;
        *ctr = 0u;
        if (ready && k0 == 0) __hip_atomic_store((gu32*)&w->ready1, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

#ifndef RS_PROBE
#define RS_PROBE 0                     // timing probes (variant builds only): 1 the fit twice, 2 rank 2 twice
#endif
#ifndef RS_WAVES_EU
#define RS_WAVES_EU 0                  // 0: the compiler's register budget
#endif
#if RS_WAVES_EU
#define RS_OCC __attribute__((amdgpu_waves_per_eu(RS_WAVES_EU)))
#else
#define RS_OCC
#endif
template <int HPB>
__global__ void __launch_bounds__(64 * HPB) RS_OCC k_ransac_hyp(VoDev d, int k0, int k1, int nhyp, int stage, int reps)
{
    ransac_chunk<HPB, RS_HYP_J, RS_HYP_PF>(d, k0, k1, nhyp, stage, reps, blockIdx.x, gridDim.x, false);
}
// one frame's two chunks in one launch (the per-frame call and the stage API: one launch and one
// dependent-launch gap less): workgroups [0, b0) run [0, c0) and publish its replay; the rest wait
// for it and run [c0, nhyp) as the second launch would
template <int HPB, bool W1>
__global__ void __launch_bounds__(64 * HPB) RS_OCC k_ransac_fused(VoDev d, int c0, int nhyp, int stage, int b0, int reps1)
{
    if ((int)blockIdx.x < b0) ransac_chunk<HPB, RS_FUSED_J, RS_FUSED_PF, W1>(d, 0, c0, nhyp, stage, 1, blockIdx.x, b0, true);
    else ransac_chunk<HPB, RS_FUSED_J, RS_FUSED_PF, W1>(d, c0, nhyp, nhyp, stage, reps1, blockIdx.x - b0, gridDim.x - b0, true);
}

// ---------------------------------------------------------------------------
// refit on the best hypothesis' inliers (model.fit(bestInlierSet), ransac.cpp:193) and the
// getPose prologue (PoseUpdate.hpp:61-96).  One wavefront; sums in the oracle's order.
// ---------------------------------------------------------------------------

// getPose prologue on w->F (PoseUpdate.hpp:64-99): E = K^T F K / |E|_F, SVD, the 4 (R, t)
// candidates; sets w->degenerate where the reference throws (PoseUpdate.hpp:71-73).  1 thread.
__device__ void pose_prep(const VoDev& d, VoWork* w)
{
    double E[9], G[9];
    mtm3(d.K, w->F, G);
    mm3(G, d.K, E);
    double nn = 0.0;
    for (int i = 0; i < 9; ++i) nn = nn + E[i] * E[i];
    nn = sqrt(nn);
    double inv = 1.0 / nn;
    int nz = 0;
    for (int i = 0; i < 9; ++i) { E[i] = E[i] * inv; nz += (E[i] != 0.0); }
    if (nz < 5) { w->degenerate = 1; return; }
    double U[9], S[3], Vt[9];
    svd3(E, U, S, Vt);
    if (det3(U) < 0) for (int i = 0; i < 9; ++i) U[i] = -U[i];
    if (det3(Vt) < 0) for (int i = 0; i < 9; ++i) Vt[i] = -Vt[i];
    const double W[9] = {0, -1, 0, 1, 0, 0, 0, 0, 1};
    const double Wt[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1};
    double R1[9], R2[9], T[9];
    mm3(U, W, T); mm3(T, Vt, R1);
    mm3(U, Wt, T); mm3(T, Vt, R2);
    if (det3(R1) < 0) for (int i = 0; i < 9; ++i) R1[i] = -R1[i];
    if (det3(R2) < 0) for (int i = 0; i < 9; ++i) R2[i] = -R2[i];
    for (int i = 0; i < 9; ++i) { w->R1[i] = R1[i]; w->R2[i] = R2[i]; }
    w->t[0] = U[2]; w->t[1] = U[5]; w->t[2] = U[8];
    w->degenerate = 0;
}

// candidate choice (PoseUpdate.hpp:142-178, first max wins) and det fix; t is the signed unit
// column before scaling
__device__ void choose_pose(const int* counts4, const double* R1, const double* R2, const double* t0, double* Rf,
                            double* tf)
{
    int maxPos = -1, bestc = 0;
    for (int c = 0; c < 4; ++c)
        if (counts4[c] > maxPos) { maxPos = counts4[c]; bestc = c; }
    const double* R = bestc < 2 ? R1 : R2;
    const double sg = (bestc & 1) ? -1.0 : 1.0;
    for (int i = 0; i < 9; ++i) Rf[i] = R[i];
    if (det3(Rf) < 0) for (int i = 0; i < 9; ++i) Rf[i] = -Rf[i];
    tf[0] = t0[0] * sg; tf[1] = t0[1] * sg; tf[2] = t0[2] * sg;
}

// t *= scale / |t| (PoseUpdate.hpp:174-177)
__device__ __forceinline__ void scale_t(double* tf, double scale)
{
    const double tn = sqrt((tf[0] * tf[0] + tf[1] * tf[1]) + tf[2] * tf[2]);
    if (tn > 1e-6) {
        const double f = scale / tn;
        tf[0] = tf[0] * f; tf[1] = tf[1] * f; tf[2] = tf[2] * f;
    }
}

// least-squares null vector (mirror of oracle ls_nullvec9): Cholesky with a pivot floor,
// W = S^-1 from the column-wise inverse of L, six power-of-two-scaled squarings to W^64, then power
// iteration from the warm start x0.  Called by the whole k_refit workgroup; each wave runs it
// (wave 1 duplicates wave 0), lanes 0..8 own rows / columns, lanes 0..44 own the upper-
// triangle entries of the squarings, and every sum runs in the oracle's ascending order.
// Returns the status (0 converged, 1 certified in the null space after the 32-step cap, 2 cyclic-
// Jacobi fallback; oracle voo_dbg_nullvec_status); f (unit) is valid in every lane.
__constant__ unsigned char c_tri9[45][2] = {
    {0, 0}, {0, 1}, {0, 2}, {0, 3}, {0, 4}, {0, 5}, {0, 6}, {0, 7}, {0, 8}, {1, 1}, {1, 2}, {1, 3},
    {1, 4}, {1, 5}, {1, 6}, {1, 7}, {1, 8}, {2, 2}, {2, 3}, {2, 4}, {2, 5}, {2, 6}, {2, 7}, {2, 8},
    {3, 3}, {3, 4}, {3, 5}, {3, 6}, {3, 7}, {3, 8}, {4, 4}, {4, 5}, {4, 6}, {4, 7}, {4, 8}, {5, 5},
    {5, 6}, {5, 7}, {5, 8}, {6, 6}, {6, 7}, {6, 8}, {7, 7}, {7, 8}, {8, 8}};

// power of two r with max_i A_ii * r in [0.5, 1) (A symmetric PSD: |A_ij| <= max_i A_ii)
__device__ __forceinline__ double pow2_scale9(const double* A)
{
    double m = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) m = A[i * 9 + i] > m ? A[i * 9 + i] : m;
    int e;
    (void)frexp(m, &e);
    return ldexp(1.0, -e);
}

// B = (rA)(rA) with r = pow2_scale9(A) (A, B symmetric 9x9 in LDS); lane e < 45 owns entry
// c_tri9[e]
__device__ __forceinline__ void sym_square9(const double* A, double* B, int lane)
{
    const double r = pow2_scale9(A);
    const int e = lane < 45 ? lane : 44;
    const int i = c_tri9[e][0], j = c_tri9[e][1];
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < 9; ++k) v = v + (A[i * 9 + k] * r) * (A[k * 9 + j] * r);
    if (lane < 45) { B[i * 9 + j] = v; B[j * 9 + i] = v; }
    __syncthreads();
}

// smallest eigenvector of the 9x9 symmetric S by cyclic Jacobi (mirror of oracle
// jacobi_min_eigvec9): one thread, a and v in LDS (a, v: 81 doubles each), f (9) to LDS.  The
// fallback of ls_nullvec9_par when its power iteration neither converges nor is certified.
__device__ __noinline__ void jacobi_min_eigvec9(const double* S, const double* x0, double* a, double* v, double* f)
{
    for (int i = 0; i < 81; ++i) { a[i] = S[i]; v[i] = (i % 10 == 0) ? 1.0 : 0.0; }
    for (int sweep = 0; sweep < 64; ++sweep) {
        int rot = 0;
        for (int p = 0; p < 8; ++p)
            for (int q = p + 1; q < 9; ++q) {
                const double apq = a[p * 9 + q];
                if (apq == 0.0) continue;
                if (fabs(apq) <= 1e-18 * (fabs(a[p * 9 + p]) + fabs(a[q * 9 + q]))) {
                    a[p * 9 + q] = 0.0; a[q * 9 + p] = 0.0;
                    continue;
                }
                ++rot;
                const double th = (a[q * 9 + q] - a[p * 9 + p]) / (2.0 * apq);
                double t = 1.0 / (fabs(th) + sqrt(th * th + 1.0));
                if (th < 0.0) t = -t;
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 9; ++k) {
                    const double akp = a[k * 9 + p], akq = a[k * 9 + q];
                    a[k * 9 + p] = c * akp - s * akq;
                    a[k * 9 + q] = s * akp + c * akq;
                }
                for (int k = 0; k < 9; ++k) {
                    const double apk = a[p * 9 + k], aqk = a[q * 9 + k];
                    a[p * 9 + k] = c * apk - s * aqk;
                    a[q * 9 + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 9; ++k) {
                    const double vkp = v[k * 9 + p], vkq = v[k * 9 + q];
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
    const double sg = dot < 0.0 ? -1.0 : 1.0;
    for (int i = 0; i < 9; ++i) f[i] = v[i * 9 + k] * sg;
}

__device__ int ls_nullvec9_par(const VoDev& d, const double* S, const double* x0, double* f, double* s_L,
                               double* s_W, double* s_W2)
{
    VO_STAMP(d, 1994, 0);
    const int lane = threadIdx.x & 63;
    const int r = lane < 9 ? lane : 8;          // row / column owned by this lane
    double mx = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i)
        if (S[i * 9 + i] > mx) mx = S[i * 9 + i];
    double fl = 1e-15 * mx;
    if (!(fl > 0.0)) fl = 1e-300;
    // Cholesky, column j: lane i computes S_ij - sum_k L_ik L_jk (lane j: the pivot)
    double Lr[9], invd[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        double v = S[r * 9 + j];
#pragma unroll
        for (int k = 0; k < j; ++k) v = v - Lr[k] * rdlane(Lr[k], j);
        double sj = rdlane(v, j);
        if (!(sj > fl)) sj = fl;
        const double dj = sqrt(sj);
        invd[j] = 1.0 / dj;
        Lr[j] = r == j ? dj : (r > j ? v * invd[j] : 0.0);
    }
    if (lane < 9) {
#pragma unroll
        for (int k = 0; k < 9; ++k) s_L[lane * 9 + k] = Lr[k];
    }
    __syncthreads();
    VO_STAMP(d, 1994, 1);
    // column c = r of L^-1 by forward substitution; the k < c terms are exact zeros
    {
        double Li[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            double v = 0.0;
#pragma unroll
            for (int k = 0; k < i; ++k) v = v + s_L[i * 9 + k] * Li[k];
            Li[i] = i < r ? 0.0 : (i == r ? invd[i] : -(v * invd[i]));
        }
        // W = L^-T L^-1 needs rows of L^-1 per entry: stage L^-1 in s_W2 (row-major)
        if (lane < 9) {
#pragma unroll
            for (int i = 0; i < 9; ++i) s_W2[i * 9 + lane] = Li[i];
        }
    }
    __syncthreads();
    {
        const int e = lane < 45 ? lane : 44;
        const int i = c_tri9[e][0], j = c_tri9[e][1];
        double v = 0.0;
        for (int k = j; k < 9; ++k) v = v + s_W2[k * 9 + i] * s_W2[k * 9 + j];
        __syncthreads();                        // all reads of L^-1 done before s_W2 is reused
        if (lane < 45) { s_W[i * 9 + j] = v; s_W[j * 9 + i] = v; }
        __syncthreads();
    }
    VO_STAMP(d, 1994, 2);
#pragma unroll 1
    for (int q = 0; q < 3; ++q) {
        sym_square9(s_W, s_W2, lane);
        sym_square9(s_W2, s_W, lane);
    }
    VO_STAMP(d, 1994, 3);
    double Wr[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) Wr[j] = s_W[r * 9 + j];
    double x[9];
    double n0 = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) n0 = n0 + x0[i] * x0[i];
    n0 = sqrt(n0);
    if (n0 > 0.0 && n0 < 1e300) {
#pragma unroll
        for (int i = 0; i < 9; ++i) x[i] = x0[i] / n0;
    } else {
#pragma unroll
        for (int i = 0; i < 9; ++i) x[i] = 1.0 / 3.0;
    }
    int it = 0;
    bool conv = false;
    for (; it < 32; ++it) {
        double zi = 0.0;
#pragma unroll
        for (int j = 0; j < 9; ++j) zi = zi + Wr[j] * x[j];
        double z[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) z[i] = rdlane(zi, i);
        double nn = 0.0, dot = 0.0;
#pragma unroll
        for (int i = 0; i < 9; ++i) { nn = nn + z[i] * z[i]; dot = dot + z[i] * x[i]; }
        nn = sqrt(nn);
        const double rs = (dot < 0.0 ? -1.0 : 1.0) / nn;
        double diff = 0.0;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const double xn = z[i] * rs;
            const double dd = fabs(xn - x[i]);
            if (dd > diff) diff = dd;
            x[i] = xn;
        }
        if (diff <= 4e-16) { ++it; conv = true; break; }
    }
    // no convergence in 32 steps (uniform over the workgroup: every lane holds the same iterate):
    // keep the iterate if its Rayleigh quotient certifies it in S's numerical null space, else
    // cyclic Jacobi on S by thread 0 in LDS (the oracle's NV_CERTIFIED / NV_JACOBI)
    int status = 0;
    if (!conv) {
        double rq = 0.0;
        for (int i = 0; i < 9; ++i) {
            double si = 0.0;
            for (int j = 0; j < 9; ++j) si = si + S[i * 9 + j] * x[j];
            rq = rq + x[i] * si;
        }
        if (rq <= 64.0 * fl) {
            status = 1;
        } else {
            status = 2;
            __syncthreads();                    // s_W / s_W2 / s_L are free: W^64 and L were read above
            if (threadIdx.x == 0) jacobi_min_eigvec9(S, x0, s_W, s_W2, s_L);
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 9; ++i) x[i] = s_L[i];
        }
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) f[i] = x[i];
    VO_STAMP(d, 1994, 4);
    return status;
}

__device__ __forceinline__ void warm_start(const double* Fb, double s1, double mx1, double my1, double s2,
                                           double mx2, double my2, double* f0)
{
    double T1i[9] = {1.0 / s1, 0.0, mx1, 0.0, 1.0 / s1, my1, 0.0, 0.0, 1.0};
    double T2i[9] = {1.0 / s2, 0.0, mx2, 0.0, 1.0 / s2, my2, 0.0, 0.0, 1.0};
    double G[9];
    mtm3(T2i, Fb, G);
    mm3(G, T1i, f0);
}

#define RF_T 128
#define RF_PCAP 512      // inlier points staged in LDS as f64 (beyond: read from L2 / HBM)
#define RF_ROWS 23       // partial-sum rows in LDS: the 45 moment sums go in two rounds
// one sum over the refit threads in the oracle's order (red_finish): per-thread partials
// -> LDS -> thread e sums the RF_T partials of quantity e as 8 sequential chains of 16,
// combined pairwise.  Quantities [E0, E0 + NS) of part, RF_ROWS at a time (42 KB of LDS in
// all: a refit workgroup fits beside the extract queue's stencil workgroups on one CU).
template <int NS, int E0 = 0, int NT = NS>
__device__ __forceinline__ void refit_sums(const double (&part)[NT], double (*s_part)[RF_T + 1], double* s_out)
{
    static_assert(NS <= RF_ROWS && E0 + NS <= NT, "refit_sums rows");
    const int tid = threadIdx.x;
#pragma unroll
    for (int e = 0; e < NS; ++e) s_part[e][tid] = part[E0 + e];
    __syncthreads();
    if (tid < NS) {
        double c[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) c[j] = 0.0;
#pragma unroll
        for (int t = 0; t < 16; ++t)
#pragma unroll
            for (int j = 0; j < 8; ++j) c[j] = c[j] + s_part[tid][16 * j + t];
        s_out[E0 + tid] = ((c[0] + c[1]) + (c[2] + c[3])) + ((c[4] + c[5]) + (c[6] + c[7]));
    }
    __syncthreads();
}

// inlier point i of the refit: LDS for i < RF_PCAP, HBM beyond
__device__ __forceinline__ void refit_pt(const double2* s_p, const double* pts, const int32_t* inl, int i, double* p)
{
    double2 a, b;
    if (i < RF_PCAP) { a = s_p[2 * i]; b = s_p[2 * i + 1]; }
    else {
        const double2* g = reinterpret_cast<const double2*>(pts + 4 * (size_t)inl[i]);
        a = g[0]; b = g[1];
    }
    p[0] = a.x; p[1] = a.y; p[2] = b.x; p[3] = b.y;
}

__global__ void __launch_bounds__(RF_T) k_refit(VoDev d, int with_pose, int stage)
{
    const int wf = blockIdx.x;                     // window frame
    if (wf >= vwin_count(d, stage)) return;
    VoWork* w = d.work + wf;
    if (w->status != VO_STATUS_OK) return;
    const double* pts = d.pts + (size_t)wf * 4 * d.N;
    int32_t* inl = d.inl + (size_t)wf * d.N;
    float* model_p = d.model_p + (size_t)wf * 4 * d.N;
    __shared__ double s_part[RF_ROWS][RF_T + 1];
    __shared__ double s_sum[45];
    __shared__ double s_A[81];
    __shared__ int s_n;
    __shared__ double2 s_p[2 * RF_PCAP];
    __shared__ uint64_t s_w[64];
    __shared__ int s_woff[64];
    const int tid = threadIdx.x, lane = tid & 63;
    const int bestk = w->bestk;
    const int scored = w->scored;
    VO_STAMP(d, 1995, 0);
    // ordered compaction of the best hypothesis' inliers from its Sampson mask (written by
    // k_ransac_hyp with the same F and test): word offsets by a wave scan, then every thread
    // places its bits; the points are staged in LDS for the three passes below
    const int nw = bestk >= 0 ? (scored + 63) >> 6 : 0;
    if (tid < 64) {
        const uint64_t mw = lane < nw ? d.inlmask[((size_t)wf * d.max_hyp + bestk) * d.mask_words + lane] : 0ull;
        const int c = __popcll(mw);
        int x = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(x, off);
            if (lane >= off) x += y;
        }
        s_w[lane] = mw;
        s_woff[lane] = x - c;
        if (lane == 63) { s_n = x; w->n_inl = x; }
    }
    __syncthreads();
    VO_STAMP(d, 1995, 1);
    const int n = s_n;
    for (int i = tid; i < nw * 64; i += RF_T) {
        const uint64_t mw = s_w[i >> 6];
        if ((mw >> (i & 63)) & 1ull) {
            const int pos = s_woff[i >> 6] + __popcll(mw & ((1ull << (i & 63)) - 1ull));
            const double2* g = reinterpret_cast<const double2*>(pts + 4 * (size_t)i);
            const double2 a = g[0], b = g[1];
            if (pos < RF_PCAP) { s_p[2 * pos] = a; s_p[2 * pos + 1] = b; }
            inl[pos] = i;
            reinterpret_cast<float4*>(model_p)[pos] = make_float4((float)a.x, (float)a.y, (float)b.x, (float)b.y);
        }
    }
    __syncthreads();
    if (bestk >= 0 && n >= 8) {
        double pm[4] = {0.0, 0.0, 0.0, 0.0};
        for (int i = tid; i < n; i += RF_T) {
            double p[4];
            refit_pt(s_p, pts, inl, i, p);
#pragma unroll
            for (int c = 0; c < 4; ++c) pm[c] = pm[c] + p[c];
        }
        refit_sums<4>(pm, s_part, s_sum);
        VO_STAMP(d, 1995, 2);
        double mean[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) mean[c] = s_sum[c] / (double)n;
        double ps[2] = {0.0, 0.0};
        for (int i = tid; i < n; i += RF_T) {
            double p[4];
            refit_pt(s_p, pts, inl, i, p);
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                double a = p[2 * g] - mean[2 * g], b = p[2 * g + 1] - mean[2 * g + 1];
                ps[g] = ps[g] + (a * a + b * b);
            }
        }
        refit_sums<2>(ps, s_part, s_sum);
        VO_STAMP(d, 1995, 3);
        const double sc1 = sqrt(2.0) / sqrt(s_sum[0] / (double)n);
        const double sc2 = sqrt(2.0) / sqrt(s_sum[1] / (double)n);
        const double o1x = -(sc1 * mean[0]), o1y = -(sc1 * mean[1]), o2x = -(sc2 * mean[2]), o2y = -(sc2 * mean[3]);
        double acc[45];
#pragma unroll
        for (int e = 0; e < 45; ++e) acc[e] = 0.0;
        for (int i = tid; i < n; i += RF_T) {
            double p[4];
            refit_pt(s_p, pts, inl, i, p);
            double a[9];
            design_row(sc1 * p[0] + o1x, sc1 * p[1] + o1y, sc2 * p[2] + o2x, sc2 * p[3] + o2y, a);
            int e = 0;
#pragma unroll
            for (int u = 0; u < 9; ++u)
#pragma unroll
                for (int v = u; v < 9; ++v) { acc[e] = acc[e] + a[u] * a[v]; ++e; }
        }
        refit_sums<23, 0>(acc, s_part, s_sum);
        refit_sums<22, 23>(acc, s_part, s_sum);
        VO_STAMP(d, 1995, 4);
        if (tid < 45) {
            int u = 0, e = tid;
            while (e >= 9 - u) { e -= 9 - u; ++u; }
            int v = u + e;
            s_A[u * 9 + v] = s_sum[tid];
            s_A[v * 9 + u] = s_sum[tid];
        }
        __syncthreads();
        double Fb[9], f0[9], f[9];
        VO_STAMP(d, 1995, 5);
        if (w->cold) {             // vo_fit_F: a plain fit, no hypothesis (oracle voo_fit_F's x0)
#pragma unroll
            for (int i = 0; i < 9; ++i) f0[i] = 1.0;
        } else {
            for (int i = 0; i < 9; ++i) Fb[i] = d.hypF[((size_t)wf * d.max_hyp + bestk) * 9 + i];
            warm_start(Fb, sc1, mean[0], mean[1], sc2, mean[2], mean[3], f0);
        }
        const int nv_status = ls_nullvec9_par(d, s_A, f0, f, &s_part[0][0], &s_part[9][0], &s_part[18][0]);
        if (tid == 0) {
            VO_STAMP(d, 1995, 6);
            w->nv_status = nv_status;
#ifdef VO_STAMPS
            if (d.dbg) d.dbg[1995 * 16 + 15] = (unsigned long long)n;
#endif
            double Fn[9];
            denormalize(f, sc1, mean[0], mean[1], sc2, mean[2], mean[3], Fn);
            rank2(Fn);
            VO_STAMP(d, 1995, 7);
            for (int i = 0; i < 9; ++i) w->F[i] = Fn[i];
            w->fitted = 1;
            w->n_fit = n;
            if (with_pose) pose_prep(d, w);
        }
    } else if (tid == 0) {
        w->fitted = 0;             // fit() returns early: the previous model stays (quirk 9)
    }
    if (tid == 0) VO_STAMP(d, 1995, 8);
}

// smallest right singular vector of the 4x4 triangulation matrix (mirror of oracle nullvec4):
// dominant eigenvector of adj(A^T A), squared four times with power-of-two scaling, then
// power-iterated from its largest-diagonal column.  One thread, no divisions but one 1/sqrt.
__device__ __forceinline__ void cof4_sym(const double* S, double* B)
{
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i; j < 4; ++j) {
            double m[9];
            int e = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (r == j) continue;
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (c != i) m[e++] = S[r * 4 + c];
            }
            double v = det3(m);
            if ((i + j) & 1) v = -v;
            B[i * 4 + j] = v; B[j * 4 + i] = v;
        }
}
__device__ __forceinline__ double pow2_scale4(const double* B)
{
    double m = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) m = B[i * 4 + i] > m ? B[i * 4 + i] : m;
    int e;
    (void)frexp(m, &e);
    return ldexp(1.0, -e);
}
__device__ __forceinline__ void nullvec4(const double* A, double* x)
{
    double S[16], B[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            S[i * 4 + j] = ((A[0 * 4 + i] * A[0 * 4 + j] + A[1 * 4 + i] * A[1 * 4 + j]) + A[2 * 4 + i] * A[2 * 4 + j]) +
                           A[3 * 4 + i] * A[3 * 4 + j];
    cof4_sym(S, B);
    double bmax = B[0];
#pragma unroll
    for (int i = 1; i < 4; ++i) bmax = B[i * 4 + i] > bmax ? B[i * 4 + i] : bmax;
    if (!(bmax > 0.0)) { x[0] = 0.0; x[1] = 0.0; x[2] = 0.0; x[3] = 1.0; return; }
#pragma unroll 1
    for (int q = 0; q < 4; ++q) {
        const double r = pow2_scale4(B);
        double B2[16];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = i; j < 4; ++j) {
                double v = 0.0;
#pragma unroll
                for (int t = 0; t < 4; ++t) v = v + (B[i * 4 + t] * r) * (B[t * 4 + j] * r);
                B2[i * 4 + j] = v; B2[j * 4 + i] = v;
            }
#pragma unroll
        for (int i = 0; i < 16; ++i) B[i] = B2[i];
    }
    int k = 0;
#pragma unroll
    for (int i = 1; i < 4; ++i) if (B[i * 4 + i] > B[k * 4 + k]) k = i;
    double y[4], nn = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double v = B[i * 4 + 0];
#pragma unroll
        for (int c = 1; c < 4; ++c) if (c == k) v = B[i * 4 + c];
        y[i] = v;
        nn = nn + y[i] * y[i];
    }
    const double rn = 1.0 / sqrt(nn);
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = y[i] * rn;
    for (int it = 0; it < 16; ++it) {
        double z[4], dot = 0.0;
        nn = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            z[i] = ((B[i * 4 + 0] * x[0] + B[i * 4 + 1] * x[1]) + B[i * 4 + 2] * x[2]) + B[i * 4 + 3] * x[3];
            nn = nn + z[i] * z[i];
            dot = dot + z[i] * x[i];
        }
        const double rs = (dot < 0.0 ? -1.0 : 1.0) / sqrt(nn);
        double diff = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const double xn = z[i] * rs;
            const double dd = fabs(xn - x[i]);
            if (dd > diff) diff = dd;
            x[i] = xn;
        }
        if (diff <= 4e-16) break;
    }
}

// cheirality test of the 4 (R, t) candidates, one thread per (refit inlier, candidate)
// (cv::undistortPoints + cv::triangulatePoints + depth test, PoseUpdate.hpp:101-147).
// grid (4N / TRI_BLOCK, B): frame wf = blockIdx.y; only frames whose own refit ran (a frame
// whose model leaked reuses the pose of the model's frame, k_finalize).
#define TRI_BLOCK 256
#ifndef TRI_BPF_DEFAULT
#define TRI_BPF_DEFAULT 8      // workgroups per frame (x 256 threads; KITTI 1.0 m/frame: 266k vs 253k frames/s for one per
                               // 128 (point, candidate) pairs; 0.05 m/frame within noise)
#endif
__device__ void finalize_body(const VoDev& d, VoFrameOut* out, int out_base);
__device__ void traj_chain(const VoDev& d, VoFrameOut* out, int out_base, int lo, int nc);
// fin: the pass's k_finalize runs in the workgroup that arrives last (every workgroup arrives,
// with or without work; the cheirality counts are agent-scope atomics, read back with agent-scope
// loads), saving the pass a launch and a queue gap
// FIN: 0 triangulation only; 1 + the pass's finalize in the last workgroup to arrive (VO_FUSE_FIN);
// 2 (the single-frame call, whose trajectory runs on the same queue) + finalize + the T_curr chain
// and pose row (k_traj's work): two launches and their gaps less per vo_process_frame
template <int FIN>
__global__ void __launch_bounds__(TRI_BLOCK) k_triangulate(VoDev d, int stage, VoFrameOut* out, int out_base)
{
    const int wf = blockIdx.y;
    VoWork* w = d.work + wf;
    __shared__ int s_cnt[4];
    __shared__ unsigned s_last;
    bool go = wf < vwin_count(d, stage);
    if (go) go = w->status == VO_STATUS_OK && w->fitted && !w->degenerate;
    const int n = go ? w->n_fit : 0;
    const unsigned active = (unsigned)((4 * n + TRI_BLOCK - 1) / TRI_BLOCK);
    go = go && blockIdx.x < active;
    if (go) {
    if (threadIdx.x < 4) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    int mycnt = 0;
    // (point, candidate) = (g >> 2, g & 3); a grid of fewer blocks than 4n / TRI_BLOCK strides
    for (int g = blockIdx.x * TRI_BLOCK + threadIdx.x; g < ((4 * n + TRI_BLOCK - 1) / TRI_BLOCK) * TRI_BLOCK;
         g += gridDim.x * TRI_BLOCK) {
    const int i = g >> 2, cnd = g & 3;
    bool pos = false;
    if (i < n) {
        const double fx = d.K[0], fy = d.K[4], cx = d.K[2], cy = d.K[5];
        const double ifx = 1.0 / fx, ify = 1.0 / fy;
        const float4 p = reinterpret_cast<const float4*>(d.model_p + (size_t)wf * 4 * d.N)[i];
        float x1 = (float)(((double)p.x - cx) * ifx), y1 = (float)(((double)p.y - cy) * ify);
        float x2 = (float)(((double)p.z - cx) * ifx), y2 = (float)(((double)p.w - cy) * ify);
        double X1 = x1, Y1 = y1, X2 = x2, Y2 = y2;
        const double* R = cnd < 2 ? w->R1 : w->R2;
        double sg = (cnd & 1) ? -1.0 : 1.0;
        double tc0 = w->t[0] * sg, tc1 = w->t[1] * sg, tc2 = w->t[2] * sg;
        double P2[12] = {R[0], R[1], R[2], tc0, R[3], R[4], R[5], tc1, R[6], R[7], R[8], tc2};
        const double P1[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        double A[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            A[0 * 4 + k] = X1 * P1[8 + k] - P1[0 + k];
            A[1 * 4 + k] = Y1 * P1[8 + k] - P1[4 + k];
            A[2 * 4 + k] = X2 * P2[8 + k] - P2[0 + k];
            A[3 * 4 + k] = Y2 * P2[8 + k] - P2[4 + k];
        }
        double X[4];
        nullvec4(A, X);
        double h0 = (double)(float)X[0], h1 = (double)(float)X[1], h2 = (double)(float)X[2], h3 = (double)(float)X[3];
        double wv = h3;
        if (!(fabs(wv) < 1e-6)) {
            double iw = 1.0 / wv;
            double Xh0 = h0 * iw, Xh1 = h1 * iw, Xh2 = h2 * iw;
            double z1 = Xh2;
            double z2 = ((R[6] * Xh0 + R[7] * Xh1) + R[8] * Xh2) + tc2;
            pos = (z1 > 0 && z2 > 0);
        }
    }
    unsigned long long bal = ballot64(pos);
    const int lane = threadIdx.x & 63;
    if (lane < 4) mycnt += __popcll(bal & (0x1111111111111111ull << lane));
    }
    if ((threadIdx.x & 63) < 4 && mycnt) atomicAdd(&s_cnt[threadIdx.x & 63], mycnt);
    __syncthreads();
    if (threadIdx.x < 4 && s_cnt[threadIdx.x])
        __hip_atomic_fetch_add((gi32*)&w->counts4[threadIdx.x], s_cnt[threadIdx.x], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (FIN == 0) return;
    if (!arrive_last(d.ctr + VO_CTR_FIN, gridDim.x * gridDim.y, &s_last)) return;
    if (threadIdx.x == 0) d.ctr[VO_CTR_FIN] = 0u;      // the next pass's launch (kernel boundary orders it)
    finalize_body(d, out, out_base);
    if constexpr (FIN == 2) {
        // k_traj: the pass log entry finalize_body wrote (this workgroup's own global stores)
        __threadfence_block();
        __syncthreads();
        const int2 lg = d.plog[d.pass % VO_PLOG];
        if (lg.y > 0) traj_chain(d, out, out_base, lg.x, lg.y);
    }
}

// lane 4q + k of each quad -> every lane of the quad (DPP quad_perm [k, k, k, k])
__device__ __forceinline__ double dpp_quad_bcast(double v, int k)
{
    const long long x = __double_as_longlong(v);
    const int lo = (int)(x & 0xFFFFFFFFll), hi = (int)(x >> 32);
    int lo2, hi2;
    switch (k) {
    case 0: lo2 = __builtin_amdgcn_update_dpp(lo, lo, 0x00, 0xF, 0xF, false); hi2 = __builtin_amdgcn_update_dpp(hi, hi, 0x00, 0xF, 0xF, false); break;
    case 1: lo2 = __builtin_amdgcn_update_dpp(lo, lo, 0x55, 0xF, 0xF, false); hi2 = __builtin_amdgcn_update_dpp(hi, hi, 0x55, 0xF, 0xF, false); break;
    case 2: lo2 = __builtin_amdgcn_update_dpp(lo, lo, 0xAA, 0xF, 0xF, false); hi2 = __builtin_amdgcn_update_dpp(hi, hi, 0xAA, 0xF, 0xF, false); break;
    default: lo2 = __builtin_amdgcn_update_dpp(lo, lo, 0xFF, 0xF, 0xF, false); hi2 = __builtin_amdgcn_update_dpp(hi, hi, 0xFF, 0xF, 0xF, false); break;
    }
    return __longlong_as_double(((long long)hi2 << 32) | (unsigned)lo2);
}

// ---------------------------------------------------------------------------
// finalize: the trajectory loop's bookkeeping over the window, in frame order
// (VisualOdometry.cpp:68-189, PoseUpdate.hpp:142-178).  One workgroup:
//   0  per frame (thread wf): its status, slots, and the pose of its own refit
//   1  thread 0: the sequential rules -- skips, missing images, the model leak (quirk 9),
//      desc1 / last_valid advance (quirk 10) -- and the commit point: the first frame after
//      a frame that did not advance desc1 was matched against the wrong previous frame, so
//      it and everything after it go to the next pass
//   2  per committed frame: the trajectory record (model R, t, kind) for k_traj, the output
//      row's counts; thread 255: the loop state and the pass log entry; all: the carry copy of
//      desc1 when the window ends in a skip (its ring slot will be rewritten)
// The T_curr chain and the pose rows run in k_traj on the trajectory queue: the next pass
// needs none of them, so they overlap it.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_finalize(VoDev d, VoFrameOut* out, int out_base)
{
    finalize_body(d, out, out_base);
}

__device__ void finalize_body(const VoDev& d, VoFrameOut* out, int out_base)
{
    constexpr int MW = VO_MAX_WIN;                    // s_R / s_t [MW]: the model before the window
    __shared__ int s_n, s_ncommit, s_lo, s_copy, s_model_wf, s_model_clear, s_newlv, s_newprev;
    __shared__ int s_status[MW], s_kind[MW], s_src[MW], s_lvb[MW];
    __shared__ int s_flip[MW], s_fitted[MW], s_degen[MW], s_cur[MW], s_adv[MW];
    __shared__ double s_R[MW + 1][9], s_t[MW + 1][3];
    __shared__ int s_rec[MW];                         // the work record each window frame uses
    __shared__ int s_dual_nc, s_dual_lend;
    const int tid = threadIdx.x;
    VO_STAMP(d, 1996, 7);
    VoState* st = d.st;
    const VoPlan P = pass_plan(d);
    const bool dual = P.dual != 0;
    if (tid == 0) {
        const int lo = st->lo;
        // a window chosen before the previous pass committed holds only if it starts where the
        // trajectory stands and its first frame was matched against the current desc1
        // (vo_internal.h VoPlan); otherwise the pass is discarded
        const int n = (P.lo == lo && P.prev0 == st->prev_slot) ? P.n : 0;
        s_lo = lo;
        s_n = n;
        s_copy = -1;
        s_model_wf = -1;
        if (dual && n > 0) {
            // repair window: frame wf > 0 uses the match against f - 1 if f - 1 advanced desc1,
            // the match against desc1 before the window if no frame before it did, else it was
            // matched against neither (the commit ends before it).  The same rules as step 1,
            // sequentially over the few frames of the window.
            bool model = st->model_n >= 8, any = false, padv = true;
            int nc = n, lend = -1;
            for (int wf = 0; wf < n; ++wf) s_rec[wf] = wf;   // frames past the commit: loaded, unused
            for (int wf = 0; wf < n; ++wf) {
                if (wf > 0 && !padv && any) { nc = wf; break; }
                const int r = (wf == 0 || padv) ? wf : n + wf;
                const VoWork* w = d.work + r;
                const bool first = w->status == VO_STATUS_FIRST, ok = w->status == VO_STATUS_OK;
                if (first) model = false;
                if (ok && w->fitted) model = true;
                const bool adv = first || (ok && model);
                s_rec[wf] = r;
                if (adv) lend = wf;
                any = any || adv;
                padv = adv;
            }
            s_dual_nc = nc;
            s_dual_lend = lend;
        }
    }
    __syncthreads();
    VO_STAMP(d, 1996, 0);
    const int n = s_n, lo = s_lo;
    if (n <= 0) {
        if (tid == 0) {
            d.plog[d.pass % VO_PLOG] = make_int2(lo, 0);   // k_traj: nothing committed
            d.snap[d.pass & (VO_PASS_RING - 1)] = VoSnap{st->lo, st->prev_slot, st->win, st->dual};
        }
        return;
    }
    // 0
    if (tid < n) {
        const VoWork* w = d.work + (dual ? s_rec[tid] : tid);
        s_status[tid] = w->status;
        s_cur[tid] = w->cur;
        const int fit = w->status == VO_STATUS_OK && w->fitted;
        s_fitted[tid] = fit;
        s_degen[tid] = w->degenerate;
        if (fit && !w->degenerate) {
            int c4[4];
            for (int c = 0; c < 4; ++c) c4[c] = ld_sc1(&w->counts4[c]);   // k_triangulate's atomics (fused: this launch)
            choose_pose(c4, w->R1, w->R2, w->t, s_R[tid], s_t[tid]);
        }
    } else if (tid == 255) {
        for (int i = 0; i < 9; ++i) s_R[MW][i] = st->model_R[i];
        for (int i = 0; i < 3; ++i) s_t[MW][i] = st->model_t[i];
    }
    __syncthreads();
    VO_STAMP(d, 1996, 1);
    // 1 (wave 0, lane = window frame of a 64-frame chunk, chunks in order with wave-uniform
    //   carries): the sequential rules as prefix operations over ballots -- the model source of
    //   a frame is its latest fit, unless a sequence start (FIRST) came after it; desc1 /
    //   last_valid advance on FIRST and on OK frames with a model; the commit stops after the
    //   first frame that did not advance (the next one was matched against it)
    if (tid < 64) {
        const int lane = tid;
        const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);   // bits <= lane
        const unsigned long long below = (1ull << lane) - 1ull;                          // bits < lane
        auto hibit = [](unsigned long long x) { return x ? 63 - __clzll((long long)x) : -1; };
        const int msrc0 = st->model_n >= 8 ? MW : -1;   // MW: the model fitted before this window
        const int mdeg = st->model_degenerate;
        const int lv0 = st->last_valid;
        int cfit = -1, cfirst = -1, cadv = -1;          // latest fit / FIRST / advance before the chunk
        int nc = n;                                     // commit: after the first frame of 0 .. n-2 that did not advance
        for (int c0 = 0; c0 < n; c0 += 64) {
            const int wf = c0 + lane;
            const bool in = wf < n;
            const int s0 = in ? s_status[wf] : -1;
            const bool first = s0 == VO_STATUS_FIRST;
            const bool ok = s0 == VO_STATUS_OK;
            const bool fitok = ok && s_fitted[wf];
            const unsigned long long Mfirst = ballot64(first), Mfit = ballot64(fitok);
            const int lf = hibit(Mfit & upto), lr = hibit(Mfirst & upto);
            const int lfit = lf >= 0 ? c0 + lf : cfit, lfirst = lr >= 0 ? c0 + lr : cfirst;
            const int msrc_l = lfit > lfirst ? lfit : (lfirst >= 0 ? -1 : msrc0);
            const int dg = msrc_l == MW ? mdeg : (msrc_l >= 0 ? s_degen[msrc_l] : 0);
            const bool okm = ok && msrc_l >= 0;
            const bool adv = first || okm;
            const unsigned long long Madv = ballot64(in && adv);
            const int la_c = hibit(Madv & below), la = la_c >= 0 ? c0 + la_c : cadv;
            if (in) {
                int o_s = s0;
                if (ok) o_s = !okm ? VO_STATUS_FEW_INLIERS : (dg ? VO_STATUS_DEGENERATE : VO_STATUS_OK);   // :147-153
                s_status[wf] = o_s;
                s_kind[wf] = (okm && !dg) ? 1 : 0;
                s_flip[wf] = (first || s0 == VO_STATUS_MISSING) ? 0 : 1;   // :58, :79 unflipped
                s_src[wf] = msrc_l;
                s_lvb[wf] = la >= 0 ? lo + la : lv0;      // :161-166 precede getPose
                s_adv[wf] = adv;
            }
            const unsigned long long nadv = ballot64(wf < n - 1 && !adv);
            if (nc == n && nadv) nc = c0 + __ffsll((long long)nadv);   // (lowest bit) + 1
            if (Mfit) cfit = c0 + hibit(Mfit);
            if (Mfirst) cfirst = c0 + hibit(Mfirst);
            if (Madv) cadv = c0 + hibit(Madv);
            if (nc < n) break;                          // later chunks are not committed
        }
        if (lane == 0) s_ncommit = dual ? s_dual_nc : nc;
    }
    __syncthreads();
    if (tid == 0) {
        // every frame before nc - 1 advanced: the last advance is nc - 1 or nc - 2 (a repair
        // window: the selection's last advance)
        const int nc = s_ncommit, prev0 = st->prev_slot, lv0 = st->last_valid;
        const int lend = dual ? s_dual_lend : (s_adv[nc - 1] ? nc - 1 : nc - 2);
        const int msrc_end = s_src[nc - 1];
        int lv = lend >= 0 ? lo + lend : lv0, prev = lend >= 0 ? s_cur[lend] : prev0;
        if (msrc_end >= 0 && msrc_end < MW) s_model_wf = msrc_end;
        s_model_clear = msrc_end < 0;                   // no model (never fitted, or a new sequence)
        if (!s_adv[nc - 1] && prev < VO_RING) { s_copy = prev; prev = VO_CARRY_SLOT; }
        s_newlv = lv; s_newprev = prev;
    }
    __syncthreads();
    VO_STAMP(d, 1996, 2);
    const int nc = s_ncommit;
    // 2
    if (tid < nc) {
        const VoWork* w = d.work + (dual ? s_rec[tid] : tid);
        const int s = s_status[tid];
        VoTrajRec* tr = d.trec + (lo + tid) % VO_RING;
        if (s_kind[tid] == 1) {
            const int src = s_src[tid];
            for (int i = 0; i < 9; ++i) tr->R[i] = s_R[src][i];
            for (int i = 0; i < 3; ++i) tr->t[i] = s_t[src][i];
        }
        tr->kind = s_kind[tid];
        tr->first = s == VO_STATUS_FIRST;
        tr->flip = s_flip[tid];
        tr->lvb = s_lvb[tid];
        VoFrameOut* o = out + (lo + tid - out_base);
        o->status = s;
        o->n_kps = s == VO_STATUS_MISSING ? 0 : d.ext_n[s_cur[tid]];
        // bit 0: this frame's select failed its check; bit 1: the context's error counter is set
        // (a bounded wait timed out somewhere: sticky until vo_reset)
        o->err = (d.ext_st[s_cur[tid]] == VO_STATUS_INCONSISTENT ? 1 : 0) |
                 (__hip_atomic_load((gu32*)(d.ctr + VO_CTR_ERR), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 2 : 0);
        o->n_matches = w->M;
        o->n_inl = w->n_inl;
        o->best_k = w->bestk;
        o->n_eval = w->n_eval;
        o->fitted = s_fitted[tid];
        o->frame = lo + tid;
    } else if (tid == 255) {
        d.plog[d.pass % VO_PLOG] = make_int2(lo, nc);
        st->lo = lo + nc;
        st->win = nc < n ? d.repair_win : d.WB;
        st->dual = nc < n && 2 * d.repair_win <= d.WB;
        st->last_valid = s_newlv;
        st->prev_slot = s_newprev;
        d.snap[d.pass & (VO_PASS_RING - 1)] = VoSnap{st->lo, st->prev_slot, st->win, st->dual};
        const int m = s_model_wf;
        if (m >= 0) {
            const VoWork* w = d.work + (dual ? s_rec[m] : m);
            st->model_n = w->n_fit;
            st->model_degenerate = s_degen[m];
            for (int i = 0; i < 9; ++i) st->model_F[i] = w->F[i];
            for (int i = 0; i < 9; ++i) st->model_R[i] = s_R[m][i];
            for (int i = 0; i < 3; ++i) st->model_t[i] = s_t[m][i];
        } else if (s_model_clear) {
            st->model_n = 0;
            st->model_degenerate = 0;
        }
    }
    VO_STAMP(d, 1996, 5);
    if (s_copy >= 0) {
        const int src = s_copy, nk = d.ext_n[src];
        const size_t N = (size_t)d.N;
        for (int i = tid; i < nk; i += blockDim.x) {
            d.kps[VO_CARRY_SLOT * N + i] = d.kps[src * N + i];
            d.pre[VO_CARRY_SLOT * N + i] = d.pre[src * N + i];
        }
        for (int i = tid; i < 8 * nk; i += blockDim.x) d.desc[VO_CARRY_SLOT * N * 8 + i] = d.desc[src * N * 8 + i];
        if (tid == 0) {
            d.ext_n[VO_CARRY_SLOT] = nk;
            d.ext_st[VO_CARRY_SLOT] = VO_STATUS_OK;
        }
    }
}

// ---------------------------------------------------------------------------
// trajectory (trajectory queue, after pass d.pass's k_finalize): the committed frames' GT scale
// and T_rel (VisualOdometry.cpp:161-166), T_curr = T_curr * T_rel in frame order (mm4's
// operation order) and the pose rows (:175-181).  One workgroup:
//   1  per committed frame: GT scale and T_rel from its trajectory record
//   2  wave 0, lane = entry: the chain, the frame kinds as wave-uniform bit masks, T_rel columns
//      read from LDS two frames ahead, so each step's critical path is the quad broadcasts and
//      the four products
//   3  per committed frame: the pose row; thread 255: T_curr
// ---------------------------------------------------------------------------
__device__ void traj_chain(const VoDev& d, VoFrameOut* out, int out_base, int lo, int nc)
{
    constexpr int MW = VO_MAX_WIN;
    __shared__ double s_Trel[MW + 2][16];             // + 2: step 2 reads two frames ahead
    __shared__ double s_row[MW][12];
    __shared__ double s_T[16];
    __shared__ int s_kind[MW], s_first[MW], s_flip[MW];
    const int tid = threadIdx.x;
    VoState* st = d.st;
    // 1
    if (tid < nc) {
        const int f = lo + tid;
        const VoTrajRec* tr = d.trec + f % VO_RING;
        const int kind = tr->kind;
        s_kind[tid] = kind;
        s_first[tid] = tr->first;
        s_flip[tid] = tr->flip;
        if (kind == 1) {
            const int lvb = tr->lvb;
            double scale = 1.0;
            if (d.gt_n > 0 && f < d.gt_n && lvb < d.gt_n) {
                double Gi[16], Gl[16], Ii[16], Tr[16];
                for (int r = 0; r < 16; ++r) {
                    Gi[r] = r < 12 ? d.gt[12 * (size_t)f + r] : (r == 15 ? 1.0 : 0.0);
                    Gl[r] = r < 12 ? d.gt[12 * (size_t)lvb + r] : (r == 15 ? 1.0 : 0.0);
                }
                inv4(Gi, Ii);
                mm4(Ii, Gl, Tr);
                scale = sqrt((Tr[3] * Tr[3] + Tr[7] * Tr[7]) + Tr[11] * Tr[11]);
            }
            double R[9], tf[3];
            for (int i = 0; i < 9; ++i) R[i] = tr->R[i];
            for (int i = 0; i < 3; ++i) tf[i] = tr->t[i];
            scale_t(tf, scale);
            double* T = s_Trel[tid];
            T[0] = R[0]; T[1] = R[1]; T[2] = R[2]; T[3] = tf[0];
            T[4] = R[3]; T[5] = R[4]; T[6] = R[5]; T[7] = tf[1];
            T[8] = R[6]; T[9] = R[7]; T[10] = R[8]; T[11] = tf[2];
            T[12] = 0.0; T[13] = 0.0; T[14] = 0.0; T[15] = 1.0;
        }
    } else if (tid == 255) {
        for (int i = 0; i < 16; ++i) s_T[i] = st->Tcurr[i];
    }
    __syncthreads();
    // 2
    if (tid < 64) {
        const int e = tid & 15, i = e >> 2, j = e & 3;
        // frame kinds of window frames 64 c + tid (chunk c) as wave-uniform masks
        constexpr int NCH = (MW + 63) / 64;
        unsigned long long Mkind[NCH], Mfirst[NCH], Mflip[NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const bool inc = 64 * c + tid < nc;
            Mkind[c] = ballot64(inc && s_kind[64 * c + tid] == 1);
            Mfirst[c] = ballot64(inc && s_first[64 * c + tid] != 0);
            Mflip[c] = ballot64(inc && s_flip[64 * c + tid] != 0);
        }
        double Tv = s_T[e];
        const double ident = (e % 5 == 0) ? 1.0 : 0.0;  // VisualOdometry.cpp:57 T_curr = eye(4)
        double b[3][4];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int k = 0; k < 4; ++k) b[u][k] = s_Trel[u][k * 4 + j];
        // branch-free: every step computes the product and selects (s_Trel rows of other
        // kinds are never used); the loads of frame wf + 2 are unconditional
        for (int wf = 0; wf < nc; ++wf) {
#pragma unroll
            for (int k = 0; k < 4; ++k) b[2][k] = s_Trel[wf + 2][k * 4 + j];
            // row i of T_curr: entry k from lane 4i + k of the quad (DPP quad broadcast)
            const double a0 = dpp_quad_bcast(Tv, 0), a1 = dpp_quad_bcast(Tv, 1);
            const double a2 = dpp_quad_bcast(Tv, 2), a3 = dpp_quad_bcast(Tv, 3);
            const double pv = ((a0 * b[0][0] + a1 * b[0][1]) + a2 * b[0][2]) + a3 * b[0][3];
            const int sh = wf & 63, ch = wf >> 6;
            unsigned long long mk = Mkind[0], mf = Mfirst[0], ml = Mflip[0];
#pragma unroll
            for (int c = 1; c < NCH; ++c)
                if (ch == c) { mk = Mkind[c]; mf = Mfirst[c]; ml = Mflip[c]; }
            const bool kind = (mk >> sh) & 1ull;
            const bool firstf = (mf >> sh) & 1ull;
            const bool flip = (ml >> sh) & 1ull;
            Tv = kind ? pv : (firstf ? ident : Tv);
            if (tid < 12) s_row[wf][tid] = (flip && i == 2) ? -Tv : Tv;
#pragma unroll
            for (int k = 0; k < 4; ++k) { b[0][k] = b[1][k]; b[1][k] = b[2][k]; }
        }
        if (tid < 16) s_T[tid] = Tv;
    }
    __syncthreads();
    // 3
    if (tid < nc) {
        VoFrameOut* o = out + (lo + tid - out_base);
        for (int r = 0; r < 12; ++r) o->pose[r] = s_row[tid][r];
    } else if (tid == 255) {
        for (int i = 0; i < 16; ++i) st->Tcurr[i] = s_T[i];
    }
}

__global__ void __launch_bounds__(256) k_traj(VoDev d, VoFrameOut* out, int out_base)
{
    // the commit point for the host (every pass's k_traj runs after its k_finalize, in pass order on
    // one queue, so the chunk's last one leaves the final value): no D2H copy after the last pass
    if (threadIdx.x == 0 && d.lo_host_dev) __hip_atomic_store(d.lo_host_dev, d.st->lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const int2 lg = d.plog[d.pass % VO_PLOG];
    if (lg.y <= 0) return;
    traj_chain(d, out, out_base, lg.x, lg.y);
}

// vo_rechain: the chain over committed frames [lo, lo + nc) (nc <= VO_MAX_WIN) from st->Tcurr,
// their trajectory records still in the ring (a sequence shard's rows from its predecessor's T_curr)
__global__ void __launch_bounds__(256) k_traj_range(VoDev d, VoFrameOut* out, int out_base, int lo, int nc)
{
    if (nc <= 0) return;
    traj_chain(d, out, out_base, lo, nc);
}

// vo_reset on the device (VisualOdometry.cpp:50-62 initial state): trajectory state, slot
// statuses, histograms, window records and cross-queue counters; no host round trip
// a frame from pinned host memory (read over PCIe by the kernel) into device memory: H2D_PT
// 16-byte loads in flight per thread, the tail bytes by the first thread
#ifndef H2D_PT
#define H2D_PT 4
#endif
__global__ void __launch_bounds__(256) k_h2d(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, size_t n)
{
    const size_t n16 = n / 16, i0 = (size_t)blockIdx.x * (256 * H2D_PT) + threadIdx.x;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    uint4 v[H2D_PT];
#pragma unroll
    for (int u = 0; u < H2D_PT; ++u)
        if (i0 + 256 * u < n16) v[u] = s4[i0 + 256 * u];
#pragma unroll
    for (int u = 0; u < H2D_PT; ++u)
        if (i0 + 256 * u < n16) d4[i0 + 256 * u] = v[u];
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (size_t i = n16 * 16; i < n; ++i) dst[i] = src[i];
}


__global__ void __launch_bounds__(256) k_reset(VoDev d)
{
    const int tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
    if (tid == 0) {
        VoState* st = d.st;
        st->lo = 0; st->end = 0; st->prev_slot = 0; st->last_valid = 0; st->win = d.WB; st->dual = 0;
        st->model_n = 0; st->model_degenerate = 0; st->pose_status = 0;
        for (int i = 0; i < 9; ++i) { st->model_F[i] = 0.0; st->model_R[i] = 0.0; st->pose_R[i] = 0.0; }
        for (int i = 0; i < 3; ++i) { st->model_t[i] = 0.0; st->pose_t[i] = 0.0; }
        for (int i = 0; i < 16; ++i) st->Tcurr[i] = (i % 5 == 0) ? 1.0 : 0.0;
        st->scale_override = __longlong_as_double(0x7FF8000000000000ll);
    }
    if (tid == 1) {
        // the pass rings as if passes d.pass - 2 and d.pass - 1 had finalized the reset state and
        // pass d.pass - 1 had an empty window: the next pass starts from the state
        const VoSnap s0{0, 0, d.WB, 0};
        d.snap[(d.pass + VO_PASS_RING - 2) & (VO_PASS_RING - 1)] = s0;
        d.snap[(d.pass + VO_PASS_RING - 1) & (VO_PASS_RING - 1)] = s0;
        d.plan[(d.pass + VO_PASS_RING - 1) & (VO_PASS_RING - 1)] = VoPlan{-1, 0, 0, -1};
    }
    for (int i = tid; i < VO_SLOTS; i += nth) { d.ext_n[i] = 0; d.ext_st[i] = VO_STATUS_OK; }
    for (int i = tid; i < VO_HIST_BINS * d.B * VO_EXT_QUEUES; i += nth) d.hist[i] = 0u;
    uint32_t* w = reinterpret_cast<uint32_t*>(d.work);
    for (int i = tid; i < (int)(sizeof(VoWork) / 4) * 2 * d.WB; i += nth) w[i] = 0u;   // both window sets
    for (int i = tid; i < VO_CTR_WORDS; i += nth) d.ctr[i] = 0u;
}

// vo_pose (PoseUpdate::getPose on caller data in work[0]): phase 0 the prologue, phase 1
// (after k_triangulate) the candidate choice and the caller's scale
__global__ void k_pose_stage(VoDev d, int phase)
{
    if (threadIdx.x != 0) return;
    VoWork* w = d.work;
    VoState* st = d.st;
    if (phase == 0) { pose_prep(d, w); return; }
    if (w->degenerate) { st->pose_status = VO_STATUS_DEGENERATE; return; }
    int c4[4];
    for (int c = 0; c < 4; ++c) c4[c] = w->counts4[c];
    double Rf[9], tf[3];
    choose_pose(c4, w->R1, w->R2, w->t, Rf, tf);
    scale_t(tf, st->scale_override);
    for (int i = 0; i < 9; ++i) st->pose_R[i] = Rf[i];
    for (int i = 0; i < 3; ++i) st->pose_t[i] = tf[i];
    st->pose_status = VO_STATUS_OK;
}

// arithmetic self-test: the ops whose rounding the parity contract depends on
__global__ void k_selftest_arith(const float* fa, const float* fb, float* fo, const double* da, const double* db,
                                 double* dout, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fo[4 * i + 0] = sqrtf(fa[i]);
    fo[4 * i + 1] = fa[i] / fb[i];
    double s, c;
    det_sincos(da[i], &s, &c);
    fo[4 * i + 2] = (float)det_atan2(da[i], db[i]);
    fo[4 * i + 3] = (float)s;
    dout[4 * i + 0] = sqrt(fabs(da[i]));
    dout[4 * i + 1] = da[i] / db[i];
    dout[4 * i + 2] = det_atan2(da[i], db[i]);
    dout[4 * i + 3] = c;
}

// null-vector solver self-test: ls_nullvec9_par on matrix b of S (one workgroup of RF_T each), as
// k_refit calls it
__global__ void __launch_bounds__(RF_T) k_selftest_nullvec9(const double* S, const double* x0, double* f, int* status)
{
    __shared__ double s_S[81], s_a[81], s_b[81], s_c[81];
    const int b = blockIdx.x;
    for (int i = threadIdx.x; i < 81; i += RF_T) s_S[i] = S[81 * b + i];
    __syncthreads();
    double x[9], out[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) x[i] = x0[9 * b + i];
    VoDev d;
    d.dbg = nullptr;
    const int st = ls_nullvec9_par(d, s_S, x, out, s_a, s_b, s_c);
    if (threadIdx.x == 0) {
        for (int i = 0; i < 9; ++i) f[9 * b + i] = out[i];
        status[b] = st;
    }
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
static const char* g_names[] = {"stencil", "select", "describe", "match", "ransac", "refit", "triangulate",
                                "finalize", "trajectory"};
int kernel_count() { return (int)(sizeof(g_names) / sizeof(g_names[0])); }
const char* kernel_name(int i) { return g_names[i]; }

// tests only (VO_FAULT_INJECT=1): N counts more in each frame's top histogram bin than the stencil
// stored keys, so the select's consistency check must fire (tests/test_gpu_parity.py
// test_select_consistency_failure_is_loud)
__global__ void k_inject_hist(VoDev d, int nb)
{
    if (threadIdx.x == 0 && (int)blockIdx.x < nb) d.hist[(size_t)blockIdx.x * VO_HIST_BINS + VO_HIST_BINS - 1] += (uint32_t)d.N;
}
// the FLAT stencil form (VO_ST_FLAT=1, NMS margins of 5+)
static bool stencil_flat(const VoDev& d)
{
    static const int flat_env = getenv("VO_ST_FLAT") ? atoi(getenv("VO_ST_FLAT")) : ST_FLAT_DEFAULT;
    return flat_env && d.brow >= 5 && d.bcol >= 5;
}
// k_select builds the batch's histogram in LDS (the stencil writes none): not with the FLAT stencil,
// nor when the LDS request leaves no room for it
static bool select_lhist(const VoDev& d)
{
    const int ntiles = ((d.W + ST_TW - 1) / ST_TW) * ((d.H + ST_TH - 1) / ST_TH);
    return ST_LHIST && !stencil_flat(d) && sel_layout(ntiles, d.sel_lds).hist >= 0;
}
// the batch's select is the one-workgroup k_select (launch_select's choice, shared so the two agree)
static bool select_single_wg(const VoDev& d, int nb)
{
    static const int sel_small = getenv("VO_SEL_SMALL") ? atoi(getenv("VO_SEL_SMALL")) : 16;
    if (d.sel1 && d.sel_emit_lds >= 0 && nb <= sel_small && !d.single) return false;
    return d.sel1 && !(d.single && d.sel_emit_lds >= 0);
}
void launch_stencil(const VoDev& d, const uint8_t* img0, size_t frame_bytes, int nb, int write_response, hipStream_t s)
{
    ensure_tables();
    const int ntx = (d.W + ST_TW - 1) / ST_TW, nsx = (ntx + 1) / 2, nty = (d.H + ST_TH - 1) / ST_TH;
    static const int segt = getenv("VO_STSEG") ? atoi(getenv("VO_STSEG")) : ST_SEGT_DEFAULT;
    // one frame (the per-frame call): segments of one tile row, so the frame's waves (4x 8-tile
    // segments' count) each walk 30 source rows instead of 142 -- the latency of the launch
    // the per-frame call's segment (VO_PF_SEGT: 1 or 2 tile rows; 2 reads 1.44x the frame's rows over
    // PCIe instead of 1.88x, in half as many waves of 46 source rows)
    static const int pf_segt = getenv("VO_PF_SEGT") && (atoi(getenv("VO_PF_SEGT")) == 2 || atoi(getenv("VO_PF_SEGT")) == 4)
                                   ? atoi(getenv("VO_PF_SEGT")) : 1;
    int st = write_response ? 4 : nb == 1 && d.single ? pf_segt
           : segt == 4 || segt == 5 || segt == 6 || segt == 8 ? segt : ST_SEGT_DEFAULT;
    // a small batch (a sequence's ragged last batch): shorter segments until the launch has two
    // waves per SIMD, since its latency is one wave's walk down its segment (8 frames at 6-tile
    // segments: 352 waves of 110 rows, 89 us; at one-tile segments 2112 waves of 30 rows)
    static const bool seg_adapt = !(getenv("VO_STSEG_ADAPT") && atoi(getenv("VO_STSEG_ADAPT")) == 0);
    if (seg_adapt && !write_response && st > 1) {
        const int steps[4] = {6, 5, 4, 1};
        for (int i = 0; i < 4 && (size_t)nb * nsx * ((nty + st - 1) / st) < 2048; ++i)
            if (steps[i] < st) st = steps[i];
    }
    // the FLAT form for NMS margins of 5+ (the reference's 35 / 37; VO_ST_FLAT=1 turns it on); the
    // general form keeps the border masks (small margins, the response map)
    const bool flat = !write_response && stencil_flat(d);
    const int waves = nsx * ((nty + st - 1) / st);             // one (strip, segment) per wave
    dim3 g(xcd_grid((waves + 3) / 4, nb));
#define ST_LAUNCH(S, F) hipLaunchKernelGGL((k_stencil<S, false, F>), g, dim3(256), 0, s, d, img0, frame_bytes, 0, nb)
#define ST_LAUNCH_NH(S) hipLaunchKernelGGL((k_stencil<S, false, false, true>), g, dim3(256), 0, s, d, img0, frame_bytes, 0, nb)
    // no histogram where k_select builds its own (ST_LHIST=0: the stencil's, as before round 6)
    const bool nh = !write_response && select_lhist(d) && select_single_wg(d, nb);
    if (write_response)
        hipLaunchKernelGGL((k_stencil<4, true, false>), g, dim3(256), 0, s, d, img0, frame_bytes, write_response, nb);
    else if (nh) {
        switch (st) {
        case 2: ST_LAUNCH_NH(2); break;
        case 4: ST_LAUNCH_NH(4); break;
        case 5: ST_LAUNCH_NH(5); break;
        case 6: ST_LAUNCH_NH(6); break;
        case 1: ST_LAUNCH_NH(1); break;
        default: ST_LAUNCH_NH(8); break;
        }
    } else if (!flat) {
        switch (st) {
        case 1: ST_LAUNCH(1, false); break;
        case 2: ST_LAUNCH(2, false); break;
        case 4: ST_LAUNCH(4, false); break;
        case 5: ST_LAUNCH(5, false); break;
        case 6: ST_LAUNCH(6, false); break;
        default: ST_LAUNCH(8, false); break;
        }
    } else {
        switch (st) {
        case 1: ST_LAUNCH(1, true); break;
        case 2: ST_LAUNCH(2, true); break;
        case 4: ST_LAUNCH(4, true); break;
        case 5: ST_LAUNCH(5, true); break;
        case 6: ST_LAUNCH(6, true); break;
        default: ST_LAUNCH(8, true); break;
        }
    }
#undef ST_LAUNCH
#undef ST_LAUNCH_NH
    if (d.fault_inject && !write_response && !nh) hipLaunchKernelGGL(k_inject_hist, dim3(nb), dim3(64), 0, s, d, nb);
}
void launch_select(const VoDev& d, int f0, int nb, int slot_override, hipStream_t s)
{
    // single frames always banded (8 workgroups, not 1); small batches too (a sequence's ragged last
    // batch, VO_SEL_SMALL frames or fewer): the one-workgroup select asks for a whole CU's LDS, so
    // under the pose queue's kernels it waits for a CU to drain (8 frames: 118 us against 25 us
    // for 64 frames alone, gpurun_out r5j), while the banded kernels' 256-thread workgroups
    // co-run.  (Whole batches keep the one-workgroup form: KITTI within noise either way.)
    static const int sel_small = getenv("VO_SEL_SMALL") ? atoi(getenv("VO_SEL_SMALL")) : 16;
    if (d.sel1 && d.sel_emit_lds >= 0 && nb <= sel_small && !d.single) {
        const dim3 g(xcd_grid(VO_SEL_BANDS, nb));
        const int cnt_lds = sel_band_layout((d.W + ST_TW - 1) / ST_TW, (d.H + ST_TH - 1) / ST_TH).bits;
        hipLaunchKernelGGL(k_select_count, g, dim3(SL_T), (size_t)cnt_lds, s, d, f0, slot_override, nb);
        hipLaunchKernelGGL(k_select_emit, g, dim3(SL_T), (size_t)d.sel_emit_lds, s, d, f0, slot_override, nb);
        return;
    }
    if (d.sel1 && !(d.single && d.sel_emit_lds >= 0)) {
        // the stencil of this batch wrote no histogram (launch_stencil's nh, the same condition)
        const int lhist = select_lhist(d) ? 1 : 0;
        hipLaunchKernelGGL(k_select, dim3(nb), dim3(1024), (size_t)d.sel_lds, s, d, f0, slot_override, lhist);
        return;
    }
    const dim3 g(xcd_grid(VO_SEL_BANDS, nb));
    if (d.single && nb == 1 && d.sel_fused) {          // the per-frame call: one launch
        const int fl = d.sel_fused == 2 ? sel_fused_lds((d.W + ST_TW - 1) / ST_TW, (d.H + ST_TH - 1) / ST_TH) : d.sel_emit_lds;
        hipLaunchKernelGGL(k_select_fused, g, dim3(SL_T), (size_t)fl, s, d, f0, slot_override, nb);
        return;
    }
    // the count kernel uses the layout's tile table only (rows, pre, tof)
    const int cnt_lds = sel_band_layout((d.W + ST_TW - 1) / ST_TW, (d.H + ST_TH - 1) / ST_TH).bits;
    hipLaunchKernelGGL(k_select_count, g, dim3(SL_T), (size_t)cnt_lds, s, d, f0, slot_override, nb);
    hipLaunchKernelGGL(k_select_emit, g, dim3(SL_T), (size_t)d.sel_emit_lds, s, d, f0, slot_override, nb);
}
int select_emit_lds_bytes(int W, int H)
{
    const int ntx = (W + ST_TW - 1) / ST_TW, nty = (H + ST_TH - 1) / ST_TH;
    const int bytes = sel_band_layout(ntx, nty).total;
    if (bytes > 150 * 1024) return -1;
    if (bytes > 64 * 1024) {
        if (hipFuncSetAttribute((const void*)k_select_emit, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess ||
            hipFuncSetAttribute((const void*)k_select_count, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess ||
            hipFuncSetAttribute((const void*)k_select_fused, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
            return -1;
    }
    return bytes;
}
int select_fused_lds_bytes(int W, int H)
{
    const int ntx = (W + ST_TW - 1) / ST_TW, nty = (H + ST_TH - 1) / ST_TH;
    const int fbytes = sel_fused_lds(ntx, nty);      // the band layout + its staged keys (96 KB)
    if (fbytes > 150 * 1024) return -1;
    if (fbytes > 64 * 1024 &&
        hipFuncSetAttribute((const void*)k_select_fused, hipFuncAttributeMaxDynamicSharedMemorySize, fbytes) != hipSuccess)
        return -1;
    return fbytes;
}
// VO_EVENT_WAIT=0: the pose queue's wait for extract batch k without an event on the extract queue
// (whose record costs that queue ~8 us between a describe and the next stencil): one wave polls the
// frame count describe's last workgroup publishes (publish_seq: every workgroup's stores released
// first), relaxed loads with a sleep between them, one acquire after; bounded like the fused
// kernels' waits (a timeout is loud: VO_CTR_ERR)
__global__ void __launch_bounds__(64) k_wait_ext(VoDev d, unsigned target)
{
    if (threadIdx.x != 0) return;
    const unsigned* c = d.ctr + VO_SYNC_EXT;
    unsigned it = 0u;
    const unsigned lim = d.spin_limit << 6;          // ~64x the fused waits' bound: a whole batch may be ahead
    while (__hip_atomic_load((gu32*)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && it < lim) {
        __builtin_amdgcn_s_sleep(8);
        ++it;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (it >= lim) atomicAdd(d.ctr + VO_CTR_ERR, 1u);
}
void launch_wait_ext(const VoDev& d, unsigned target, hipStream_t s)
{
    hipLaunchKernelGGL(k_wait_ext, dim3(1), dim3(64), 0, s, d, target);
}
void launch_ext_missing(const VoDev& d, int slot, hipStream_t s)
{
    hipLaunchKernelGGL(k_ext_missing, dim3(1), dim3(64), 0, s, d, slot);
}
int select_lds_bytes(int W, int H, int* key_cap)
{
    const int ntiles = ((W + ST_TW - 1) / ST_TW) * ((H + ST_TH - 1) / ST_TH);
    // the whole CU's LDS: keys staged in LDS are read 4 times (a 64 KB request, which lets other
    // kernels share the CU, measured 2-3 % slower end to end)
    // VO_SEL_LDS_KB: a smaller request (the keys then stay in global scratch past its capacity)
    static const int kb = getenv("VO_SEL_LDS_KB") ? std::max(40, std::min(158, atoi(getenv("VO_SEL_LDS_KB")))) : 158;
    const int bytes = kb == 158 ? 160 * 1024 - 2048 : kb * 1024;   // static __shared__ of k_select < 2 KB
    if (hipFuncSetAttribute((const void*)k_select, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
        return -1;
    const SelLayout L = sel_layout(ntiles, bytes);
    if (L.key_cap < 1024) return -1;
    if (key_cap) *key_cap = L.key_cap;
    return bytes;
}
void launch_describe(const VoDev& d, int f0, int nb, int slot_override, unsigned publish, hipStream_t s)
{
    ensure_tables();
    // VO_DS_LDS_TABLE=1: the per-frame call's describe reads the pair table from LDS (measured: describe
    // 26 -> 30 us, the call 165 -> 168 us, so the scalar-cache path stays the default)
    static const int lt_env = getenv("VO_DS_LDS_TABLE") ? atoi(getenv("VO_DS_LDS_TABLE")) : 0;
    // (the batched describe with the LDS table, measured round 6: KITTI 280.6-281.5k vs 297.7-302.5k,
    // describe 0.96 -> 1.11 us/frame, r6t)
    const bool lt = lt_env != 0 && nb == 1 && d.single;
    // the per-frame call: eight waves per 64 keypoints (VO_DS_PF=0: one, k_describe)
    static const int pf_env = getenv("VO_DS_PF") ? atoi(getenv("VO_DS_PF")) : 1;
    if (pf_env && nb == 1 && d.single && !publish && !lt) {
        hipLaunchKernelGGL(k_describe_pf, dim3((d.N + 63) / 64), dim3(64 * DP_WAVES), 0, s, d, f0, slot_override);
        return;
    }
    if (lt)
        hipLaunchKernelGGL(k_describe<true>, dim3(xcd_grid((d.N + DS_KPB - 1) / DS_KPB, nb)), dim3(64 * DS_WAVES), 0, s, d,
                           f0, slot_override, publish, nb);
    else
        hipLaunchKernelGGL(k_describe<false>, dim3(xcd_grid((d.N + DS_KPB - 1) / DS_KPB, nb)), dim3(64 * DS_WAVES), 0, s,
                           d, f0, slot_override, publish, nb);
}
// the kernel symbol(s) (base names, comma-separated) stage k of the batched path launches for
// this context -- what a rocprofv3 summary of the same run lists (bench.py profile_row)
const char* kernel_form(const VoDev& d, int k)
{
    switch (k) {
    case 0: return "k_stencil";
    case 1: return d.sel1 ? "k_select" : "k_select_count,k_select_emit";
    case 2: return "k_describe";
    case 3: return d.match_bits == 32 ? "k_match" : "k_match512";
    case 4: return "k_ransac_hyp";
    case 5: return "k_refit";
    case 6: return "k_triangulate";
    case 7: return "k_finalize";
    case 8: return "k_traj";
    }
    return "";
}
void launch_match(const VoDev& d, int stage, hipStream_t s)
{
    if (d.match_bits == 32) {
        // single-frame calls: one query per lane (4x the workgroups, a quarter of the walk each)
        if (d.single)
            hipLaunchKernelGGL((k_match<1, MT_SINGLE_WAVES>), dim3((d.N + 63) / 64, stage ? 1 : d.gridw),
                               dim3(64 * MT_SINGLE_WAVES), 0, s, d, stage);
        else
            hipLaunchKernelGGL(k_match<MT_QPL>, dim3(match_blocks(d.N, 32), stage ? 1 : d.gridw), dim3(256), 0, s, d, stage);
    } else {
        // 64 KB of dynamic LDS plus the static hand-off words: above the default 64 KB cap
        static const bool lds_ok = hipFuncSetAttribute((const void*)k_match512,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       MT512_TILE * 64) == hipSuccess;
        (void)lds_ok;
        hipLaunchKernelGGL(k_match512, dim3(match_blocks(d.N, 512), stage ? 1 : d.gridw), dim3(256),
                           (size_t)MT512_TILE * 64, s, d, stage);
    }
}
// hypotheses in three chunks, [0, C0), [C0, C1), [C1, max_hyp): a frame's later chunks exit at
// once when its replay has already stopped (ransac.cpp:139 adaptive bound; 100 hypotheses for
// most frames).  One wave per hypothesis, four per workgroup: with B frames per launch there
// are enough hypotheses to fill the chip, so no wave repeats another's 8-point fit.
void launch_ransac(const VoDev& d, int stage, hipStream_t s, int part)
{
    const int nhyp = d.max_hyp, nb = stage ? 1 : d.gridw;
    // (the per-frame call's window: one frame, two work records -- the repair form's second record)
    if (part == 0 && (stage || d.single) && nb <= 2 && d.ransac_fused && nhyp > VO_HYP_CHUNK0) {
        // one hypothesis per wave (4 per workgroup), the wave's lanes splitting its count: the count's
        // latency is 7 Sampson tests per lane instead of 52 (VO_RANSAC_WAVE_HYP=0: eight hypotheses per
        // wave, 32 per workgroup).  (Round 5 also measured four waves splitting one eight-hypothesis
        // set's count through LDS: slower, 138-140 vs 136.7 us per call.)
        static const bool w1 = !(getenv("VO_RANSAC_WAVE_HYP") && atoi(getenv("VO_RANSAC_WAVE_HYP")) == 0);
        const int hpg = w1 ? 4 : 32;
        const int b0 = (VO_HYP_CHUNK0 + hpg - 1) / hpg, b1 = (nhyp - VO_HYP_CHUNK0 + hpg - 1) / hpg;
        // the later chunk on at most 60 workgroups (hypothesis blocks strided by the grid): its
        // workgroups wait for the first chunk's replay, and hundreds of pollers slowed it
        static const int wg1 = getenv("VO_RANSAC_WG1") ? std::max(1, atoi(getenv("VO_RANSAC_WG1"))) : 60;
        const int n1 = std::min(b1, wg1), reps1 = (b1 + n1 - 1) / n1;
        if (w1) hipLaunchKernelGGL((k_ransac_fused<4, true>), dim3(b0 + n1, nb), dim3(256), 0, s, d, VO_HYP_CHUNK0, nhyp, stage, b0, reps1);
        else hipLaunchKernelGGL((k_ransac_fused<4, false>), dim3(b0 + n1, nb), dim3(256), 0, s, d, VO_HYP_CHUNK0, nhyp, stage, b0, reps1);
        return;
    }
    // the cuts after [0, VO_HYP_CHUNK0): VO_HYP_CHUNK1 (VO_HYP_CUTS: a list, ascending, e.g. "400,700"; "0"
    // or a cut >= max_hyp merges every later chunk into one)
    static const std::vector<int> cuts_env = [] {
        std::vector<int> v;
        const char* e = getenv("VO_HYP_CUTS");
        if (!e) { v.push_back(VO_HYP_CHUNK1); return v; }
        for (const char* q = e; *q;) {
            const int x = atoi(q);
            if (x > VO_HYP_CHUNK0 && (v.empty() || x > v.back())) v.push_back(x);
            while (*q >= '0' && *q <= '9') ++q;
            if (*q) ++q;                          // any one separator (',' or ':')
        }
        return v;
    }();
    int cut[16], nc = 0;
    cut[nc++] = std::min(nhyp, VO_HYP_CHUNK0);
    for (int x : cuts_env)
        if (x < nhyp && nc < 15) cut[nc++] = x;
    cut[nc++] = nhyp;
    int k0 = 0;
    for (int c = 0; c < nc; ++c) {
        const int k1 = cut[c];
        if (k1 <= k0) continue;
        if ((part == 1 && c > 0) || (part == 2 && c == 0)) { k0 = k1; continue; }
        static const int r2 = getenv("VO_RREPS") ? std::max(1, atoi(getenv("VO_RREPS"))) : VO_HYP_REPS;
        const int reps = c == 0 ? 1 : (c < nc - 1 ? std::max(1, r2 / 2) : r2);
        const int blocks = ((k1 - k0 + 31) / 32 + reps - 1) / reps;      // 32 hypotheses per workgroup
        hipLaunchKernelGGL((k_ransac_hyp<4>), dim3(blocks, nb), dim3(256), 0, s, d, k0, k1, nhyp, stage, reps);
        k0 = k1;
    }
}
void launch_refit(const VoDev& d, int with_pose, int stage, hipStream_t s)
{
    hipLaunchKernelGGL(k_refit, dim3(stage ? 1 : d.gridw), dim3(RF_T), 0, s, d, with_pose, stage);
}
void launch_triangulate(const VoDev& d, int stage, hipStream_t s, VoFrameOut* out, int out_base, int fin)
{
    // blocks per frame (VO_TRI_BPF; 0 = one (point, candidate) per thread, 4N / TRI_BLOCK blocks)
    static const int bpf_env = getenv("VO_TRI_BPF") ? atoi(getenv("VO_TRI_BPF")) : TRI_BPF_DEFAULT;
    const int full = (4 * d.N + TRI_BLOCK - 1) / TRI_BLOCK;
    const int bpf = bpf_env > 0 ? std::min(bpf_env, full) : full;
    const dim3 g(bpf, stage ? 1 : d.gridw);
    if (fin == 2) hipLaunchKernelGGL(k_triangulate<2>, g, dim3(TRI_BLOCK), 0, s, d, stage, out, out_base);
    else if (fin) hipLaunchKernelGGL(k_triangulate<1>, g, dim3(TRI_BLOCK), 0, s, d, stage, out, out_base);
    else hipLaunchKernelGGL(k_triangulate<0>, g, dim3(TRI_BLOCK), 0, s, d, stage, out, out_base);
}
void launch_finalize(const VoDev& d, VoFrameOut* out, int out_base, hipStream_t s)
{
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(256), 0, s, d, out, out_base);
}
void launch_traj(const VoDev& d, VoFrameOut* out, int out_base, hipStream_t s)
{
    hipLaunchKernelGGL(k_traj, dim3(1), dim3(256), 0, s, d, out, out_base);
}

void launch_traj_range(const VoDev& d, VoFrameOut* out, int out_base, int lo, int nc, hipStream_t s)
{
    hipLaunchKernelGGL(k_traj_range, dim3(1), dim3(256), 0, s, d, out, out_base, lo, nc);
}
void launch_h2d(uint8_t* dst, const uint8_t* src, size_t n, hipStream_t s)
{
    const size_t n16 = n / 16;
    const int blocks = (int)std::max<size_t>(1, (n16 + H2D_PT * 256 - 1) / (H2D_PT * 256));
    hipLaunchKernelGGL(k_h2d, dim3(blocks), dim3(256), 0, s, dst, src, n);
}
void launch_reset(const VoDev& d, hipStream_t s)
{
    hipLaunchKernelGGL(k_reset, dim3(16), dim3(256), 0, s, d);
}
void launch_pose_stage(const VoDev& d, int phase, hipStream_t s)
{
    hipLaunchKernelGGL(k_pose_stage, dim3(1), dim3(64), 0, s, d, phase);
}
void launch_selftest_nullvec9(const double* S, const double* x0, double* f, int* status, int n, hipStream_t s)
{
    hipLaunchKernelGGL(k_selftest_nullvec9, dim3(n), dim3(RF_T), 0, s, S, x0, f, status);
}
void launch_selftest_arith(const float* fa, const float* fb, float* fo, const double* da, const double* db,
                           double* dout, int n, hipStream_t s)
{
    hipLaunchKernelGGL(k_selftest_arith, dim3((n + 255) / 256), dim3(256), 0, s, fa, fb, fo, da, db, dout, n);
}

}  // namespace vo

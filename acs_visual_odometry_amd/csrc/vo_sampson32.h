// f32 certificate for the Sampson inlier test of RANSAC's count (computeSampsonError(F, m) < 1,
// ransac.cpp:12-23,163-166) -- the decision the f64 chain of sampson_inlier makes, taken in f32
// wherever an error bound proves it, and left to the f64 chain (exactly as before) where it
// cannot.  Counts, masks and best hypotheses stay bit-identical; the f32 form just costs a third of
// the f64 one's instructions and latency (two matches per packed instruction).
//
// The f64 test (sampson_inlier, thr = 1): with the f64 linear forms
//   Fx0 = F0 x + F1 y + F2,  Fx1 = F3 x + F4 y + F5                       (frame-1 point x, y)
//   Ft0 = F0 x' + F3 y' + F6, Ft1 = F1 x' + F4 y' + F7, Ft2 = F2 x' + F5 y' + F8   (frame-2 x', y')
//   v = Ft0 x + Ft1 y + Ft2,  num = v^2,  den = ((Fx0^2 + Fx1^2) + Ft0^2) + Ft1^2
// the match is an inlier iff den >= 1e-12 and num < den.
//
// The f32 evaluation (f = f32(F), coordinates rounded to f32, every step one fma or product) is
// compared to the f64 one through a bound B on |num32 - num64| + |den32 - den64| that holds for every
// match of the hypothesis, built from per-hypothesis magnitudes (|x| <= X, |y| <= Y, |x'| <= X',
// |y'| <= Y': the frame's coordinate bounds, VoWork.cmax), u = 2^-24:
//   S(Fx0) = |F0| X + |F1| Y + |F2| (and alike), each linear form within e = 8u S of the f64 one (f32:
//     F and coordinate rounding plus two fma roundings, at most 4u S; f64: 3 * 2^-53 S);
//   v within ev = 4u (T0 X + T1 Y + T2) + e(Ft0) X + e(Ft1) Y + e(Ft2), T = S(Ft)(1 + 8u);
//   |num32 - num64| <= 2 ev |v| + 2 ev^2 + 2u num32;
//   |den32 - den64| <= sum_i e_i (2 S_i (1 + 8u) + e_i) + 8u den32;
// so B = K0 + K1 |v| + K2 (num + den) with K0 = 2 (KD + 2 ev^2) + 1e-30, K1 = 4 ev, K2 = 16u (the
// factor 2 and the K2 slack absorb the roundings of B and of num - den themselves, the 1e-30 any
// f32 underflow).  Then
//   num - den < -B  and  den - B > 1.01e-12   =>  inlier (num64 < den64, den64 >= 1e-12),
//   num - den > B                              =>  outlier,
//   otherwise (a match within the bound of the threshold, or a NaN / inf anywhere) the f64 test.
// tests/test_sampson32.py checks the certificate against the f64 test on the bench's hypotheses
// and on matches placed at the threshold (host build of this header: g++ with fmaf); the GPU parity
// tests check every count.
#ifndef VO_SAMPSON32_H
#define VO_SAMPSON32_H

#include <math.h>

#ifdef __HIPCC__
#define VO_S32_HD __host__ __device__
#else
#define VO_S32_HD
#endif

struct VoS32 {
    float f[9];          // f32(F)
    float k0, k1, k2;    // B = k0 + k1 |v| + k2 (num + den)
    int ok;              // every constant finite (else: the f64 test for every match)
};

// one hypothesis' constants (in f64, rounded up to f32); cm = (X, Y, X', Y')
VO_S32_HD inline void vo_s32_setup(const double* F, const float* cm, VoS32* s)
{
    const double u = 5.9604644775390625e-08;   // 2^-24
    const double cL = 8.0 * u;
    const double X = cm[0], Y = cm[1], Xp = cm[2], Yp = cm[3];
    double a[9];
    for (int i = 0; i < 9; ++i) a[i] = fabs(F[i]);
    const double S0 = a[0] * X + a[1] * Y + a[2];      // Fx0
    const double S1 = a[3] * X + a[4] * Y + a[5];      // Fx1
    const double T0 = a[0] * Xp + a[3] * Yp + a[6];    // Ft0
    const double T1 = a[1] * Xp + a[4] * Yp + a[7];    // Ft1
    const double T2 = a[2] * Xp + a[5] * Yp + a[8];    // Ft2
    const double e0 = cL * S0, e1 = cL * S1, et0 = cL * T0, et1 = cL * T1, et2 = cL * T2;
    const double g = 1.0 + cL;
    const double ev = 4.0 * u * (T0 * g * X + T1 * g * Y + T2 * g) + et0 * X + et1 * Y + et2;
    const double KD = e0 * (2.0 * S0 * g + e0) + e1 * (2.0 * S1 * g + e1) + et0 * (2.0 * T0 * g + et0) +
                      et1 * (2.0 * T1 * g + et1);
    const double up = 1.0 + 1.0 / 1048576.0;            // round the constants up past f32 rounding
    const double K0 = (2.0 * (KD + 2.0 * ev * ev) + 1e-30) * up;
    const double K1 = 4.0 * ev * up;
    for (int i = 0; i < 9; ++i) s->f[i] = (float)F[i];
    s->k0 = (float)K0;
    s->k1 = (float)K1;
    s->k2 = (float)(16.0 * u);
    // finite constants (no overflow to inf in f32), finite F
    bool ok = K0 < 1e30 && K1 < 1e30 && S0 < 1e30 && S1 < 1e30 && T0 < 1e30 && T1 < 1e30 && T2 < 1e30;
    s->ok = ok ? 1 : 0;
}

// decision of one match (or two, T = a 2-vector of float on the device): +1 inlier, 0 outlier,
// -1 undecided.  Fma and Abs are the element-wise fma and |.| of T.
template <class T, class Fma, class Abs>
VO_S32_HD inline void vo_s32_eval(const VoS32& s, T x, T y, T xp, T yp, Fma fma_, Abs abs_, T* diff, T* bnd, T* den)
{
    const T f0 = (T)s.f[0], f1 = (T)s.f[1], f2 = (T)s.f[2], f3 = (T)s.f[3], f4 = (T)s.f[4], f5 = (T)s.f[5],
            f6 = (T)s.f[6], f7 = (T)s.f[7], f8 = (T)s.f[8];
    const T fx0 = fma_(f0, x, fma_(f1, y, f2));
    const T fx1 = fma_(f3, x, fma_(f4, y, f5));
    const T ft0 = fma_(f0, xp, fma_(f3, yp, f6));
    const T ft1 = fma_(f1, xp, fma_(f4, yp, f7));
    const T ft2 = fma_(f2, xp, fma_(f5, yp, f8));
    const T v = fma_(ft0, x, fma_(ft1, y, ft2));
    const T n = v * v;
    const T d = fma_(ft1, ft1, fma_(ft0, ft0, fma_(fx1, fx1, fx0 * fx0)));
    *bnd = fma_((T)s.k1, abs_(v), fma_((T)s.k2, n + d, (T)s.k0));
    *diff = n - d;
    *den = d;
}

// the threshold of the degenerate-denominator test, above 1e-12 by more than f32 rounding
#define VO_S32_DEN_MIN 1.01e-12f

VO_S32_HD inline int vo_s32_decide(float diff, float bnd, float den)
{
    if (diff < -bnd && den - bnd > VO_S32_DEN_MIN) return 1;
    if (diff > bnd) return 0;
    return -1;
}

#endif

// Host check of the f32 Sampson certificate (acs_visual_odometry_amd/csrc/vo_sampson32.h) against the
// f64 test it stands for (sampson_inlier, thr = 1: computeSampsonError < 1, ransac.cpp:12-23).
// Usage: sampson32_check <F.bin: n x 9 f64> <pts.bin: m x 4 f64> <W> <H>   (W = 0: bounds from the points,
// as the stage API computes them).  Every hypothesis against every match; prints
// "inlier outlier undecided wrong" and the first wrong cases.  Built with -ffp-contract=off: the f64
// chain is the kernels' and the oracle's, operation for operation.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "vo_sampson32.h"

static bool f64_inlier(const double* F, double x, double y, double xp, double yp)
{
    double Fx0 = (F[0] * x + F[1] * y) + F[2] * 1.0;
    double Fx1 = (F[3] * x + F[4] * y) + F[5] * 1.0;
    double Ft0 = (F[0] * xp + F[3] * yp) + F[6] * 1.0;
    double Ft1 = (F[1] * xp + F[4] * yp) + F[7] * 1.0;
    double Ft2 = (F[2] * xp + F[5] * yp) + F[8] * 1.0;
    double v = (Ft0 * x + Ft1 * y) + Ft2 * 1.0;
    double num = v * v;
    double den = ((Fx0 * Fx0 + Fx1 * Fx1) + Ft0 * Ft0) + Ft1 * Ft1;
    if (den < 1e-12) return 1.7976931348623157e308 < 1.0;
    return num < den;
}

static std::vector<double> load(const char* p)
{
    std::vector<double> v;
    FILE* f = std::fopen(p, "rb");
    if (!f) return v;
    double x;
    while (std::fread(&x, sizeof(double), 1, f) == 1) v.push_back(x);
    std::fclose(f);
    return v;
}

int main(int argc, char** argv)
{
    if (argc < 5) return 2;
    const std::vector<double> F = load(argv[1]), P = load(argv[2]);
    const double W = std::atof(argv[3]), H = std::atof(argv[4]);
    const size_t nF = F.size() / 9, m = P.size() / 4;
    float cm[4];
    if (W > 0) { cm[0] = (float)W; cm[1] = (float)H; cm[2] = (float)W; cm[3] = (float)H; }
    else {
        double mx[4] = {0, 0, 0, 0};
        for (size_t i = 0; i < m; ++i)
            for (int k = 0; k < 4; ++k) {
                const double v = P[4 * i + k];
                mx[k] = std::isfinite(v) ? std::fmax(mx[k], std::fabs(v)) : HUGE_VAL;
            }
        for (int k = 0; k < 4; ++k) {
            float f = (float)mx[k];
            if ((double)f < mx[k]) f = std::nextafter(f, HUGE_VALF);
            cm[k] = f;
        }
    }
    const auto fma1 = [](float a, float b, float c) { return std::fmaf(a, b, c); };
    const auto abs1 = [](float a) { return std::fabs(a); };
    long long nin = 0, nout = 0, nund = 0, nwrong = 0, notok = 0;
    for (size_t h = 0; h < nF; ++h) {
        VoS32 s;
        vo_s32_setup(&F[9 * h], cm, &s);
        if (!s.ok) { ++notok; nund += (long long)m; continue; }
        for (size_t i = 0; i < m; ++i) {
            const double* p = &P[4 * i];
            float diff, bnd, den;
            vo_s32_eval(s, (float)p[0], (float)p[1], (float)p[2], (float)p[3], fma1, abs1, &diff, &bnd, &den);
            const int dcs = vo_s32_decide(diff, bnd, den);
            if (dcs < 0) { ++nund; continue; }
            const bool ref = f64_inlier(&F[9 * h], p[0], p[1], p[2], p[3]);
            (dcs ? nin : nout) += 1;
            if ((dcs == 1) != ref) {
                if (nwrong < 10)
                    std::printf("WRONG h=%zu i=%zu dec=%d ref=%d diff=%.9g bnd=%.9g den=%.9g\n", h, i, dcs, (int)ref,
                                (double)diff, (double)bnd, (double)den);
                ++nwrong;
            }
        }
    }
    std::printf("%lld %lld %lld %lld %lld\n", nin, nout, nund, nwrong, notok);
    return 0;
}

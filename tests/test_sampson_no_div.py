"""Device shortcut in the Sampson inlier test (sampson_inlier in vo_kernels.hip): for the
reference threshold 1.0 (VisualOdometry.cpp:130) and den >= 1e-12, RN(num/den) < 1 <=> num < den.
Proof sketch: num < den => num <= den - ulp(den) => num/den <= 1 - 2^-53, representable, so the
rounded quotient stays < 1; num >= den => quotient >= 1.  Checked here on random and
boundary operands, including NaN / inf."""
import numpy as np


def test_num_lt_den_equals_rounded_quotient_lt_one():
    rng = np.random.default_rng(0)
    den = np.exp(rng.uniform(np.log(1e-12), np.log(1e12), 2_000_000))
    rel = rng.choice([0.0, 1.0, -1.0, 2.0, -2.0, 1e-17, -1e-17], den.size) * 2.0 ** -53
    num = den * (1.0 + rel)
    num = np.concatenate([num, np.nextafter(den, 0), np.nextafter(den, np.inf), den])
    den = np.concatenate([den, den, den, den])
    q = num / den
    assert np.array_equal(q < 1.0, num < den)
    # num = v*v and den = sum of squares: num in [0, inf] or NaN, den >= 1e-12, inf or NaN
    specials = np.array([np.nan, np.inf, 0.0, 1e-300, 1e300])
    for a in specials:
        for b in [1e-12, 1.0, 1e300, np.inf, np.nan]:
            with np.errstate(all="ignore"):
                assert (np.float64(a) / np.float64(b) < 1.0) == (np.float64(a) < np.float64(b)), (a, b)

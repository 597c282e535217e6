"""The slip draw compares integers (rmx_internal.h slip_threshold, rmx_device.h slip_choice): numpy's
Generator.random() is u = m * 2^-53 with m = next64 >> 11, and cdf <= u exactly when ceil(cdf * 2^53) <= m.
Checked here on the values where the two could part: cdf on, just below and just above the 2^-53 grid."""
import math

import numpy as np


def threshold(cdf):  # restates slip_threshold
    if cdf != cdf:
        return (1 << 64) - 1
    if cdf <= 0.0:
        return 0
    if cdf >= 1.0:
        return (1 << 53) + (1 if cdf > 1.0 else 0)
    return int(math.ceil(math.ldexp(cdf, 53)))


def test_integer_threshold_equals_float_compare():
    rng = np.random.default_rng(5)
    ms = [0, 1, 2, (1 << 53) - 1, (1 << 52)] + [int(x) for x in rng.integers(0, 1 << 53, 200, dtype=np.int64)]
    cdfs = [0.0, -0.0, 1.0, 1.0000000000000002, 0.1, 0.9, 0.1 + 0.8, 2 ** -53, 2 ** -54, float("nan"), -1.0]
    for m in ms[:60]:
        u = m * 2.0 ** -53
        cdfs += [u, np.nextafter(u, 0.0), np.nextafter(u, 1.0)]
    cdfs += [float(c) for c in rng.random(200)]
    for c in cdfs:
        t = threshold(float(c))
        for m in ms:
            u = m * 2.0 ** -53  # exact: m < 2^53
            assert (float(c) <= u) == (t <= m), (c, m)

#!/usr/bin/env python3
"""Check of the step kernel's FMA order decode (csrc/imenv_device.h decode_orders, IMENV_DECODE_FMA)
against the reference's float64 expression (IM_env.py:298-302, MAIM_env.py:340-347):

    reference  o = clip(rint((x - a) * c))            x float32 promoted to float64, c = om / (b - a)
    kernel     o = clamp(sat_int(rint(fma(x, c, -a * c))), 0, om)

for a in {0, -1}, integral c (1 <= c <= 2^24), float32 x: every float32 within 64 ulps of each
rounding boundary (k + 1/2) / c + a, the tiny and huge magnitudes, +-0, +-inf, NaN, and random
float32 values. The FMA is emulated exactly (Fraction, then one rounding to float64).

    python tools/check_decode_fma.py
"""
import math
import random
from fractions import Fraction

import numpy as np


def ref(x, a, c, om, clip_round):
    v = (x - a) * c                     # float64, two roundings as the reference
    if clip_round:
        return int(np.rint(min(max(v, 0.0), om))) if not math.isnan(v) else 0
    r = np.rint(v)
    return int(min(max(r, 0.0), om)) if not math.isnan(r) else 0


def fma(x, y, z):
    if any(math.isinf(t) or math.isnan(t) for t in (x, y, z)):
        return x * y + z
    return float(Fraction(x) * Fraction(y) + Fraction(z))


def kern(x, a, c, om):
    v = fma(x, float(c), -a * c)
    if math.isnan(v):
        return 0
    r = np.rint(v)
    k = int(max(min(r, 2**31 - 1), -2**31))   # v_cvt_i32_f64 saturates
    return min(max(k, 0), om)


def f32_neighbours(v, n):
    x = np.float32(v)
    out = [x]
    up = dn = x
    for _ in range(n):
        up = np.nextafter(up, np.float32(np.inf))
        dn = np.nextafter(dn, np.float32(-np.inf))
        out += [up, dn]
    return [float(t) for t in out]


def check(cases=((-1.0, 15, 30), (-1.0, 1, 2), (-1.0, 3, 6), (0.0, 5, 5), (-1.0, 50, 100), (0.0, 7, 7)),
          n_rand=20000, seed=0):
    rng = random.Random(seed)
    bad, n = [], 0
    for a, c, om in cases:
        xs = [0.0, -0.0, math.inf, -math.inf, math.nan, 1e-45, -1e-45, 2.0**-30, -2.0**-30, 2.0**-29,
              3e38, -3e38, 2.0**53, -2.0**53]
        for k in range(-2, 2 * om + 3):
            xs += f32_neighbours((k + 0.5) / c + a, 64)
        xs += [float(np.float32(rng.uniform(-1.5, 1.5))) for _ in range(n_rand)]
        xs += [float(np.float32(rng.uniform(-1, 1) * 10.0 ** rng.randint(-40, 38))) for _ in range(n_rand // 4)]
        for x in xs:
            for cr in (False, True):
                n += 1
                r, k = ref(x, a, c, om, cr), kern(x, a, c, om)
                if r != k:
                    bad.append((a, c, om, cr, x, r, k))
    return n, bad


if __name__ == "__main__":
    n, bad = check()
    for b in bad[:10]:
        print("MISMATCH", b)
    print(n, "cases", len(bad), "mismatches")
    raise SystemExit(1 if bad else 0)

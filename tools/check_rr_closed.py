#!/usr/bin/env python3
"""Exhaustive check of the two-child closed-form round robin (csrc/imenv_device.h rr_closed<2>) against
the reference's literal loop (IM_div_env.py:413-498): final counts, shipments, amount left and guard
outcome, over x0, x1 in [-4, 13], amt in [-2, 31], 8 guard limits, with and without the sum check.

    python tools/check_rr_closed.py
"""
import itertools


def literal(x, s, amt, lim, sumcheck):
    """The reference's loop: while [sum(x) > 0 and] amt > 0, one unit to every child with x > 0; the
    guard raises after lim rounds (the state at that point is returned with ok = False)."""
    x = list(x)
    s = list(s)
    rounds = 0
    while (not sumcheck or sum(x) > 0) and amt > 0:
        if x[0] <= 0 and x[1] <= 0:
            # no child eligible: every further round changes nothing, so the loop spins until the guard
            # (taken in one jump: a 2^30 guard limit would otherwise loop 2^30 times here)
            return x, s, amt, False
        for k in range(2):
            if x[k] > 0:
                s[k] += 1
                x[k] -= 1
                amt -= 1
        rounds += 1
        if rounds > lim:
            return x, s, amt, False
    return x, s, amt, True


def i32(v):
    """C int32 wrap-around (the kernel's int arithmetic)."""
    return ((v + 2 ** 31) % 2 ** 32) - 2 ** 31


def closed(x, s, amt, lim, sumcheck):
    """rr_closed<2> statement by statement (C int32 semantics: >> is arithmetic, lim + 1 wraps)."""
    x0, x1 = x
    s0, s1 = s
    go1 = amt > 0 and (not sumcheck or x0 + x1 > 0)
    r1 = min(min(min(x0, x1), (amt + 1) >> 1), i32(lim + 1))
    if not (go1 and x0 > 0 and x1 > 0):
        r1 = 0
    x0 -= r1
    x1 -= r1
    s0 += r1
    s1 += r1
    amt -= 2 * r1
    e0, e1 = x0 > 0, x1 > 0
    go2 = go1 and amt > 0 and r1 <= lim
    r2 = min(x0 if e0 else (x1 if e1 else 0), amt)
    if sumcheck:
        r2 = min(r2, x0 + x1)
    r2 = min(r2, i32(i32(lim + 1) - r1))
    r2 = max(r2, 0) if go2 else 0
    r2a = r2 if e0 else 0
    r2b = r2 - r2a
    x0 -= r2a
    s0 += r2a
    x1 -= r2b
    s1 += r2b
    amt -= r2
    trip = go2 and not sumcheck and amt > 0
    return [x0, x1], [s0, s1], amt, (r1 + r2 <= lim and not trip)


def check(xr=range(-4, 14), ar=range(-2, 32), lims=(0, 1, 2, 3, 5, 8, 13, 60)):
    n = 0
    bad = []
    for x0, x1 in itertools.product(xr, xr):
        for amt in ar:
            for lim in lims:
                for sc in (True, False):
                    for s in ([0, 0], [3, 1]):
                        n += 1
                        a = literal((x0, x1), s, amt, lim, sc)
                        b = closed((x0, x1), s, amt, lim, sc)
                        if a != b:
                            bad.append(((x0, x1, amt, lim, sc, s), a, b))
    return n, bad


if __name__ == "__main__":
    n, bad = check()
    for b in bad[:10]:
        print("MISMATCH", *b)
    print(n, "cases", len(bad), "mismatches")
    raise SystemExit(1 if bad else 0)

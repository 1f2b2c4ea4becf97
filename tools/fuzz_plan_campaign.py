#!/usr/bin/env python3
"""GPU-vs-oracle campaign for the plan replay (imenv_plan_rollout) over many drawn configurations
(GPU box; tests/test_plan_gpu.py runs 8 of them as tests). Each case: tests/test_plan_gpu.py's
drawn_plan_case (all four classes, capacities 5-450, shared or per-episode plans, float32 or float64,
in-kernel demand, noisy demand / delay), 2 plans x 293 scenarios, every per-episode value and per-step
reward compared bit for bit. Prints a progress line every 50 cases and a JSON summary; exits 1 on
any mismatch.

    python tools/fuzz_plan_campaign.py [--cases 400] [--start 200000]
"""
import argparse
import json
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "marl-for-im_amd"), os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=400)
    ap.add_argument("--start", type=int, default=200000)
    args = ap.parse_args()
    import test_plan_gpu as tp
    bad, t0 = [], time.time()
    kinds = {}
    for k in range(args.cases):
        seed = args.start + k
        try:
            got, ref, kind = tp.drawn_plan_case(seed, k)
            kinds[kind] = kinds.get(kind, 0) + 1
            diff = [f for f in tp.STATS + ("rewards",) if not np.array_equal(got[f], ref[f])]
            if diff:
                bad.append(dict(case=seed, kind=kind, fields=diff))
                print("MISMATCH case %d (%s): %s" % (seed, kind, diff), flush=True)
        except Exception:
            bad.append(dict(case=seed, error=traceback.format_exc()[-400:]))
            print("ERROR case %d" % seed, flush=True)
            traceback.print_exc()
        if (k + 1) % 50 == 0:
            print("%d cases, %d bad, %.0f s" % (k + 1, len(bad), time.time() - t0), flush=True)
    print(json.dumps(dict(cases=args.cases, start=args.start, kinds=kinds, bad=len(bad), failures=bad[:20],
                          seconds=round(time.time() - t0, 1))), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

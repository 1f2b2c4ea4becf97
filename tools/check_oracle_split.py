#!/usr/bin/env python3
"""The oracle's two split modes on the large-capacity drawn tree cases of tools/fuzz_gpu_campaign.py --big
(capacities ~20,000-60,000): the reference's literal unit-by-unit round robin (oracle split="literal") and
the phase-at-a-time form (split="closed") the GPU campaign uses there, compared on every state, info,
observation, reward and guard flag of whole episodes. CPU only (the build container); a pool of worker
processes; one JSON summary line.

    python tools/check_oracle_split.py [--start 850000] [--cases 200] [--envs 8] [--procs 4]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def one(args):
    i, E = args
    import numpy as np
    import fuzz_gpu_campaign as fc
    import test_oracle_golden as tog
    from oracle.im_oracle import OracleEnv
    meta, d = fc.make_big_case(i, E)
    if not meta["kind"].endswith("div"):
        return None
    res, secs = {}, {}
    for mode in ("closed", "literal"):
        tog.OracleEnv = lambda kind, cfg, n_envs=1, m=mode: OracleEnv(kind, cfg, n_envs=n_envs, split=m)
        t0 = time.time()
        o0, out, env = tog.run_oracle(meta, d)
        secs[mode] = time.time() - t0
        res[mode] = (o0, out, env.err.copy())
    a, b = res["closed"], res["literal"]
    same = (np.array_equal(a[0], b[0]) and all(np.array_equal(a[1][k], b[1][k]) for k in a[1])
            and np.array_equal(a[2], b[2]))
    return dict(case=i, kind=meta["kind"], equal=bool(same), closed_s=round(secs["closed"], 3),
                literal_s=round(secs["literal"], 1), trips=int(a[2].astype(bool).sum()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=int, default=850000)
    ap.add_argument("--cases", type=int, default=200)
    ap.add_argument("--envs", type=int, default=8)
    ap.add_argument("--procs", type=int, default=4)
    a = ap.parse_args()
    t0 = time.time()
    with mp.get_context("fork").Pool(a.procs) as pool:
        rows = [r for r in pool.imap(one, [(a.start + k, a.envs) for k in range(a.cases)]) if r is not None]
    bad = [r for r in rows if not r["equal"]]
    for r in rows:
        print(json.dumps(r), flush=True)
    print(json.dumps(dict(start=a.start, cases=a.cases, tree_cases=len(rows), mismatches=len(bad), bad=bad[:10],
                          literal_s_total=round(sum(r["literal_s"] for r in rows), 1),
                          closed_s_total=round(sum(r["closed_s"] for r in rows), 2),
                          envs_with_guard_trips=sum(r["trips"] for r in rows), seconds=round(time.time() - t0, 1))))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

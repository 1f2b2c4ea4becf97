#!/usr/bin/env python3
"""GPU-vs-oracle campaign over drawn specifications with drawn demand (IMENV_LAYOUT_DRAW: in-kernel Philox,
Poisson or uniform, noisy demand on trees), two episodes each: the drawn-demand hand-over forced on with
the hipRTC kernel, and forced off with the ahead-of-time kernel (tests/test_drawn_fuzz_gpu.py runs 16 of
these cases as tests). The oracle runs the split closed-form (pinned equal to the literal loops by
tests/test_split_closed_form.py). Prints a progress line every 25 cases and a JSON summary; exits 1 on
any mismatch; --budget stops before a case would pass the time limit.

    python tools/fuzz_drawn_campaign.py [--cases 200] [--start 1000] [--budget SECONDS]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "marl-for-im_amd"), os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402


def run_case(i, dtab, kernel):
    import torch
    from imenv import VectorInvEnv
    from oracle.im_oracle import OracleEnv
    from test_drawn_fuzz_gpu import make_drawn_case, rng_of
    os.environ["IMENV_DTAB"] = dtab
    kind, cfg, n = make_drawn_case(i)
    off = 37 * i
    env = VectorInvEnv(kind, cfg, n_envs=n, device=torch.device("cuda:0"), env_offset=off)
    try:
        env.set_jit(1 if kernel == "jit" else 0)
        assert (env.draw_layout() > 0) == (dtab == "1")
        ora = OracleEnv(kind, cfg, n_envs=n, split="closed")
        rs = np.random.RandomState(i)
        for ep in range(2):
            env.reset()
            ora.reset(rng=rng_of(cfg, ep, off))
            for t in range(env.T):
                a = rs.uniform(-1.2, 1.2, size=(n, env.N))
                o_g, r_g, _, _ = env.step(torch.as_tensor(a, device="cuda:0"))
                o_c, r_c, _, _ = ora.step(a)
                if not (np.array_equal(o_g.cpu().numpy(), o_c.astype(np.float32))
                        and np.array_equal(r_g.cpu().numpy(), r_c)):
                    return "mismatch ep %d t %d" % (ep, t)
            st = env.state()
            for k in ("inv", "backlog", "order_u"):
                if not np.array_equal(st[k].cpu().numpy(), ora.state_arrays()[k]):
                    return "state %s mismatch ep %d" % (k, ep)
        if ("jit:" in env.kernel_info()) != (kernel == "jit"):
            return "kernel %s" % env.kernel_info()
        return None
    finally:
        env.close()
        os.environ.pop("IMENV_DTAB", None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=200)
    ap.add_argument("--start", type=int, default=1000)
    ap.add_argument("--budget", type=float, default=None)
    a = ap.parse_args()
    t0 = time.time()
    done, bad, per = 0, [], []
    for i in range(a.start, a.start + a.cases):
        if a.budget and per and time.time() - t0 + 2 * max(per) > a.budget:
            break
        c0 = time.time()
        for dtab, kernel in (("1", "jit"), ("0", "aot")):
            err = run_case(i, dtab, kernel)
            if err:
                bad.append({"case": i, "dtab": dtab, "kernel": kernel, "error": err})
                print("MISMATCH", bad[-1], flush=True)
        per.append(time.time() - c0)
        done += 1
        if done % 25 == 0:
            print("%d cases, %d mismatches, %.0f s" % (done, len(bad), time.time() - t0), flush=True)
    print(json.dumps({"cases": done, "runs": 2 * done, "start": a.start, "mismatches": bad,
                      "seconds": round(time.time() - t0, 1)}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""GPU-vs-oracle campaign over many drawn specifications (GPU box; tests/test_fuzz_gpu.py runs 32 of
them as tests). Each case: a drawn configuration (tests/fuzz_configs.py, capacities 5-450, explicit
order_max), 32 envs, host demand and float64 actions, noisy delay with host uniforms in some; the
whole episode is compared with the oracle bit for bit (state, info, float64 obs, rewards). Prints a
progress line every 50 cases and a JSON summary; exits 1 on any mismatch.

    python tools/fuzz_gpu_campaign.py [--cases 400] [--start 100000] [--mode jit|aot|both] [--big --envs 8]
                                      [--split literal|closed] [--literal-every K] [--budget SECONDS]

--big draws capacities of ~20,000-60,000, where the oracle's literal round-robin split loops for minutes
per case; there the oracle runs the same loops phase by phase (--split closed, the default with --big;
pinned equal to the literal loops by tests/test_split_closed_form.py), and every K-th case also runs the
literal loops and compares the two oracles. --budget stops before a case would pass the time limit, so
the campaign always ends with its JSON summary.
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


def make_big_case(i, E):
    """test_fuzz_gpu.make_case with the largest capacity scale of tests/fuzz_configs.py."""
    from fuzz_configs import fuzz_inputs, maybe_order_max, rand_config
    rs = np.random.RandomState(i)
    kind = ["IM", "MAIM", "IM_div", "MAIM_div"][i % 4]
    cfg = maybe_order_max(rs, kind, rand_config(rs, kind, 4))
    noisy = 0.3 if rs.rand() < 0.3 else 0.0
    dem, act, unif = fuzz_inputs(kind, cfg, {}, i, E)
    meta = dict(kind=kind, config=cfg, noisy=noisy, E=E, T=cfg["num_periods"])
    return meta, dict(customer_demand=dem, actions=act, delay_uniforms=unif if noisy else np.zeros((0,)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=400)
    ap.add_argument("--start", type=int, default=100000)
    ap.add_argument("--mode", default="both", choices=["jit", "aot", "both"])
    ap.add_argument("--envs", type=int, default=32)
    ap.add_argument("--big", action="store_true",
                    help="capacities ~20,000-60,000 (int32 state rows; the oracle's split loop is slow: few envs)")
    ap.add_argument("--split", choices=["literal", "closed"], default=None,
                    help="the oracle's split loops (default: closed with --big, else literal)")
    ap.add_argument("--literal-every", type=int, default=0,
                    help="also run the literal split on every K-th tree case and compare the oracles (0: never)")
    ap.add_argument("--budget", type=float, default=0.0, help="stop before this many seconds (0: no limit)")
    args = ap.parse_args()
    import test_fuzz_gpu as tf
    import test_gpu_parity as tp
    import test_oracle_golden as tog
    from oracle.im_oracle import OracleEnv
    split = args.split or ("closed" if args.big else "literal")

    def run_oracle(meta, d, mode=split):
        tog.OracleEnv = lambda kind, cfg, n_envs=1: OracleEnv(kind, cfg, n_envs=n_envs, split=mode)
        return tog.run_oracle(meta, d)
    os.environ["IMENV_JIT_STRICT"] = "1"
    tf.E = args.envs
    bad, t0, done = [], time.time(), 0
    keys = ["order", "demand", "acquisition", "ship", "inv", "backlog", "order_u", "profit", "obs"]
    trees, literal_checked, slowest = 0, 0, 0.0
    for k in range(args.cases):
        if args.budget and time.time() - t0 + 2 * slowest > args.budget:
            print("budget: stopping after %d cases (slowest case %.0f s)" % (done, slowest), flush=True)
            break
        c0 = time.time()
        i = args.start + k
        mode = args.mode if args.mode != "both" else ("jit" if k % 2 == 0 else "aot")
        try:
            meta, d = make_big_case(i, args.envs) if args.big else tf.make_case(i)
            obs0_o, out_o, env_o = run_oracle(meta, d)
            if meta["kind"].endswith("div"):
                trees += 1
            if (args.literal_every and split == "closed" and meta["kind"].endswith("div")
                    and (trees - 1) % args.literal_every == 0):
                # the phase-at-a-time oracle against the literal loops on this case (slow at big capacities)
                obs0_l, out_l, env_l = run_oracle(meta, d, "literal")
                if not (np.array_equal(obs0_l, obs0_o) and all(np.array_equal(out_l[q], out_o[q]) for q in out_o)
                        and np.array_equal(env_l.err, env_o.err)):
                    bad.append(dict(case=i, mode="oracle", kind=meta["kind"], fields=["closed vs literal split"]))
                    print("MISMATCH case %d: closed vs literal oracle split" % i, flush=True)
                literal_checked += 1
            tp.MODE["kernel"] = mode
            obs0_g, out_g, anyerr = tp.run_gpu_case(meta, d)
            diff = []
            if anyerr != 0 or env_o.err.any():
                diff.append("split-guard flags")
            if not np.array_equal(obs0_g, obs0_o):
                diff.append("obs0")
            for key in keys + (["ship_to", "backlog_to"] if meta["kind"].endswith("div") else []):
                if not np.array_equal(out_g[key].astype(np.float64), out_o[key]):
                    diff.append(key)
            if not np.array_equal(out_g["reward"], out_o["reward"]):
                diff.append("reward")
            if diff:
                bad.append(dict(case=i, mode=mode, kind=meta["kind"], fields=diff))
                print("MISMATCH case %d (%s, %s): %s" % (i, mode, meta["kind"], diff), flush=True)
        except Exception:
            bad.append(dict(case=i, mode=mode, error=traceback.format_exc()[-400:]))
            print("ERROR case %d (%s)" % (i, mode), flush=True)
            traceback.print_exc()
        done += 1
        slowest = max(slowest, time.time() - c0)
        if done % 50 == 0 or args.big:      # a big tree case takes the oracle ~1 min: report each
            print("%d cases, %d bad, %.0f s" % (done, len(bad), time.time() - t0), flush=True)
    print(json.dumps(dict(cases=done, start=args.start, mode=args.mode, envs=args.envs, big=args.big,
                          oracle_split=split, tree_cases=trees, literal_split_checked=literal_checked,
                          mismatches=len(bad), bad=bad[:20], seconds=round(time.time() - t0, 1),
                          slowest_case_s=round(slowest, 1))))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

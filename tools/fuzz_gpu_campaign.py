#!/usr/bin/env python3
"""GPU-vs-oracle campaign over many drawn specifications (GPU box; tests/test_fuzz_gpu.py runs 32 of
them as tests). Each case: a drawn configuration (tests/fuzz_configs.py, capacities 5-450, explicit
order_max), 32 envs, host demand and float64 actions, noisy delay with host uniforms in some; the
whole episode is compared with the oracle bit for bit (state, info, float64 obs, rewards). Prints a
progress line every 50 cases and a JSON summary; exits 1 on any mismatch.

    python tools/fuzz_gpu_campaign.py [--cases 400] [--start 100000] [--mode jit|aot|both] [--big --envs 8]
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
    args = ap.parse_args()
    import test_fuzz_gpu as tf
    import test_gpu_parity as tp
    from test_oracle_golden import run_oracle
    os.environ["IMENV_JIT_STRICT"] = "1"
    tf.E = args.envs
    bad, t0, done = [], time.time(), 0
    keys = ["order", "demand", "acquisition", "ship", "inv", "backlog", "order_u", "profit", "obs"]
    for k in range(args.cases):
        i = args.start + k
        mode = args.mode if args.mode != "both" else ("jit" if k % 2 == 0 else "aot")
        try:
            meta, d = make_big_case(i, args.envs) if args.big else tf.make_case(i)
            obs0_o, out_o, env_o = run_oracle(meta, d)
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
        if done % 50 == 0 or args.big:      # a big tree case takes the oracle ~1 min: report each
            print("%d cases, %d bad, %.0f s" % (done, len(bad), time.time() - t0), flush=True)
    print(json.dumps(dict(cases=done, start=args.start, mode=args.mode, envs=args.envs, mismatches=len(bad),
                          bad=bad[:20], seconds=round(time.time() - t0, 1))))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

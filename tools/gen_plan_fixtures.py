#!/usr/bin/env python3
"""Golden vectors for the open-loop plan replay, produced by the REFERENCE's own env classes.

Runs only in the build container (the reference is mounted read-only at /root/reference). For each
case it runs the LP scripts' evaluation loop (SHLP_8.py:737-766; the same loop in SHLP_div1.py:570-597
and the other LP / Oracle scripts) on the reference env, literally:

    s = env.reset(customer_demand=demand[j])
    while not done:
        s, r, done, info = env.step(plan[t])
        profit[j, t] = r
        total_inventory += sum(s[:, 0]); total_backlog += sum(s[:, 1]); customer_backlog += s[0, 1]
        lp_reward += r

with LP-like plans (non-integral orders, values just below / above integers, negatives, orders above
capacity), every case with standardise_state False as the LP scripts configure it. Output:
tests/golden/plan_replay.npz (data only).

    python tools/gen_plan_fixtures.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_fixtures import OUT, REF, div1, div2, import_reference, jsonable, serial4, serial8  # noqa: E402

RAW = dict(standardise_state=False, standardise_actions=False)
CASES = {
    # name: (kind, config, layout, P plans, S scenarios)
    "SHLP8": ("IM", serial8(**RAW), "episode", 1, 8),                       # SHLP_8.py DFO_CONFIG
    "SHLP4": ("IM", serial4(**RAW), "episode", 2, 6),
    "SHLP_div1": ("IM_div", div1(**RAW), "episode", 1, 8),                  # SHLP_div1.py LP_CONFIG
    "SHLP_div2": ("IM_div", div2(**RAW), "episode", 1, 6),
    "IM4_shared": ("IM", serial4(**RAW), "shared", 3, 6),
    "IM4_stdact_shared": ("IM", serial4(standardise_state=False), "shared", 2, 5),
    "div1_shared": ("IM_div", div1(**RAW), "shared", 2, 4),
}


def fuzz_cases(num=4):
    """Drawn single-agent configurations (tests/fuzz_configs.py) with raw state, as the LP scripts."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
    from fuzz_configs import maybe_order_max, rand_config
    rs = np.random.RandomState(4242)
    out = {}
    for i in range(num):
        kind = ("IM", "IM_div")[i % 2]
        cfg = maybe_order_max(rs, kind, rand_config(rs, kind, (i // 2) % 4))
        cfg["standardise_state"] = False
        top = float(np.max(cfg["inv_max"]))
        cfg.update(demand_dist="poisson", mu=float(np.round(rs.uniform(0.05, 0.5) * top, 1)))
        out["fz%d_%s" % (i, kind)] = (kind, cfg, ("episode", "shared")[i % 2], 2, 4)
    return out


def lp_like_plan(rs, shape, order_max, std):
    """Plans as an LP solver returns them: mostly integral values with float noise of either sign,
    some half-integers, a few negatives and values above order_max (the env clips and rounds)."""
    if std:
        return rs.uniform(-1.3, 1.3, size=shape)
    base = rs.randint(0, int(order_max.max()) + 6, size=shape).astype(np.float64)
    noise = rs.choice([0.0, 1e-9, -1e-9, 1e-7, 0.5, -0.5, 0.49999999], size=shape)
    plan = base + noise
    plan[rs.rand(*shape) < 0.05] = -rs.uniform(0, 3)
    return plan


def main():
    if not os.path.isdir(REF):
        print("reference not mounted; nothing to do (fixtures are committed)")
        return
    classes = import_reference()
    out, meta = {}, {}
    for ci, (name, (kind, cfg, layout, P, S)) in enumerate(list(CASES.items()) + list(fuzz_cases().items())):
        rs = np.random.RandomState(700 + ci)
        env = classes[kind](dict(cfg))
        N = env.num_nodes if hasattr(env, "num_nodes") else env.num_stages
        R = len(env.retailers) if hasattr(env, "retailers") else 1
        T = env.num_periods
        mu = cfg.get("mu", 5)
        dem = rs.poisson(mu, size=(S, R, T))
        dem = dem[:, 0, :] if kind == "IM" else dem
        std = bool(cfg.get("standardise_actions", True))
        om = np.asarray(env.order_max, dtype=np.float64)
        plans = lp_like_plan(rs, (T, P, S, N) if layout == "episode" else (P, T, N), om, std)
        ret = np.zeros((P, S))
        inv = np.zeros((P, S))
        bl = np.zeros((P, S))
        cbl = np.zeros((P, S))
        rew = np.zeros((T, P, S))
        for p in range(P):
            for j in range(S):
                env.reset(customer_demand=dem[j].copy())
                lp_reward = 0
                total_inventory = 0
                total_backlog = 0
                customer_backlog = 0
                done = False
                t = 0
                while not done:
                    action = plans[t, p, j] if layout == "episode" else plans[p, t]
                    s, r, done, info = env.step(np.array(action))
                    rew[t, p, j] = r
                    total_inventory += sum(s[:, 0])
                    total_backlog += sum(s[:, 1])
                    customer_backlog += s[0, 1]
                    lp_reward += r
                    t += 1
                ret[p, j] = lp_reward
                inv[p, j] = total_inventory
                bl[p, j] = total_backlog
                cbl[p, j] = customer_backlog
        out[name + "/plans"] = plans
        out[name + "/demand"] = dem.astype(np.int64)
        out[name + "/return"] = ret
        out[name + "/inventory"] = inv
        out[name + "/backlog"] = bl
        out[name + "/customer_backlog"] = cbl
        out[name + "/rewards"] = rew
        meta[name] = dict(kind=kind, config=jsonable(cfg), layout=layout)
        print("%-18s %-7s %-7s P=%d S=%d return[0,0]=%r" % (name, kind, layout, P, S, ret[0, 0]))
    out["meta"] = json.dumps(meta)
    np.savez_compressed(os.path.join(OUT, "plan_replay.npz"), **out)


if __name__ == "__main__":
    main()

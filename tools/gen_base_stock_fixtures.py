#!/usr/bin/env python3
"""Golden vectors for the base-stock rollout, produced by the REFERENCE's own code.

Runs only in the build container (the reference is mounted read-only at /root/reference). It
imports base_restock_policy.py and the env classes (same stand-ins as tools/gen_fixtures.py) and
records, per case, what the reference computes for P policies x S demand rows:

  objective   base_restock_policy.dfo_func(policy, env, demand)            (:24-45)
  rewards     per-step rewards of the same episode stepped with base_stock_policy (:4-21)
  return      sum of the rewards, as the evaluation loop does (inv_management.py:222-232)
  inventory / backlog / customer_backlog   sums of env.inv / env.backlog[1..T] (harness metrics)

plus one optimize_inventory_policy run (Powell from 25s on the first demand row,
inv_management.py:217-218). Output: tests/golden/base_stock.npz (data only).

    python tools/gen_base_stock_fixtures.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_fixtures import OUT, REF, div1, div2, import_reference, jsonable, serial4, serial8  # noqa: E402

NONSTD = dict(standardise_state=False, standardise_actions=False)
CASES = {
    # name: (kind, config, P policies, S demand rows, demand mean)
    "IM4_dfo": ("IM", serial4(**NONSTD), 6, 16, 5),
    "IM4_dfo_mu12": ("IM", serial4(**NONSTD), 4, 12, 12),
    "IM4_std": ("IM", serial4(), 3, 8, 5),
    "IM4_uniform": ("IM", serial4(demand_dist="uniform", lower_upper=(1, 5), **NONSTD), 4, 8, None),
    "IM8_dfo": ("IM", serial8(**NONSTD), 4, 8, 5),
    "IM_div1_dfo": ("IM_div", div1(**NONSTD), 4, 8, 5),
    "IM_div2_dfo": ("IM_div", div2(**NONSTD), 3, 6, 5),
}


def fuzz_cases(num=8):
    """Drawn single-agent configurations (tests/fuzz_configs.py) for dfo_func: IM and IM_div, raw or
    standardised actions, Poisson or uniform demand at the capacity's scale, the objective's
    retailer rows x periods within the kernel's pairwise-sum block (R * T <= 128)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
    from fuzz_configs import maybe_order_max, rand_config
    rs = np.random.RandomState(31337)
    out = {}
    for i in range(num):
        kind = ("IM", "IM_div")[i % 2]
        while True:
            cfg = maybe_order_max(rs, kind, rand_config(rs, kind, (i // 2) % 4))
            R = sum(1 for v in cfg["connections"].values() if not v) if kind == "IM_div" else 1
            if R * cfg["num_periods"] <= 128:
                break
        top = float(np.max(cfg["inv_max"]))
        if i % 3 == 2:
            lo = int(rs.randint(0, max(2, int(top // 4))))
            cfg.update(demand_dist="uniform", lower_upper=(lo, lo + 2 + int(rs.randint(0, max(2, int(top // 2))))))
            mu = None
        else:
            mu = float(np.round(rs.uniform(0.05, 0.5) * top, 1))
            cfg.update(demand_dist="poisson", mu=mu)
        out["fz%d_%s" % (i, kind)] = (kind, cfg, 3, 4, mu)
    return out


def policies_for(N, P, rs, top=60.0):
    pol = [np.ones(N) * 25.0, np.arange(1, N + 1) * 10.0]
    while len(pol) < P:
        pol.append(rs.uniform(0.0, top, size=N))      # non-integral levels, some above capacity
    return np.array(pol[:P])


def main():
    if not os.path.isdir(REF):
        print("reference not mounted; nothing to do (fixtures are committed)")
        return
    classes = import_reference()
    import base_restock_policy as brp      # the reference module (on sys.path via import_reference)

    out = {}
    meta = {}
    for ci, (name, (kind, cfg, P, S, mu)) in enumerate(list(CASES.items()) + list(fuzz_cases().items())):
        rs = np.random.RandomState(420 + ci)
        env = classes[kind](dict(cfg))
        N = env.num_nodes if hasattr(env, "num_nodes") else env.num_stages
        R = len(env.retailers) if hasattr(env, "retailers") else 1
        T = env.num_periods
        if mu is None:
            lo, hi = cfg["lower_upper"]
            dem = rs.randint(lo, hi, size=(S, R, T))
        else:
            dem = rs.poisson(mu, size=(S, R, T))
        dem = dem[:, 0, :] if kind == "IM" else dem
        pol = policies_for(N, P, rs, 60.0 if not name.startswith("fz") else 1.5 * float(np.max(cfg["inv_max"])))
        obj = np.zeros((P, S))
        rew = np.zeros((P, S, T))
        ret = np.zeros((P, S))
        inv = np.zeros((P, S))
        bl = np.zeros((P, S))
        cbl = np.zeros((P, S))
        retailers = list(env.retailers) if hasattr(env, "retailers") else [0]
        for p in range(P):
            for s in range(S):
                obj[p, s] = brp.dfo_func(pol[p], env, dem[s])
                env.reset(customer_demand=dem[s])
                r_sum = 0
                done = False
                t = 0
                while not done:
                    a = brp.base_stock_policy(pol[p], env)
                    _, r, done, _ = env.step(a)
                    rew[p, s, t] = r
                    r_sum += r
                    t += 1
                ret[p, s] = r_sum
                inv[p, s] = env.inv[1:T + 1].sum()
                bl[p, s] = env.backlog[1:T + 1].sum()
                cbl[p, s] = env.backlog[1:T + 1][:, retailers].sum()
        out[name + "/policies"] = pol
        out[name + "/demand"] = dem.astype(np.int64)
        out[name + "/objective"] = obj
        out[name + "/rewards"] = rew
        out[name + "/return"] = ret
        out[name + "/inventory"] = inv
        out[name + "/backlog"] = bl
        out[name + "/customer_backlog"] = cbl
        meta[name] = dict(kind=kind, config=jsonable(cfg))
        print("%-14s %-7s P=%d S=%d obj[0,0]=%r" % (name, kind, P, S, obj[0, 0]))

    # Powell search from 25s on the first demand row (inv_management.py:217-218)
    kind, cfg = "IM", serial4(**NONSTD)
    env = classes[kind](dict(cfg))
    d0 = out["IM4_dfo/demand"][0]
    policy, res = brp.optimize_inventory_policy(env, brp.dfo_func, init_policy=np.ones(4) * 25, demand=d0)
    out["powell/demand"] = d0
    out["powell/policy"] = np.asarray(policy, dtype=np.int64)
    out["powell/x"] = np.asarray(res.x, dtype=np.float64)
    out["powell/fun"] = np.array(float(res.fun))
    out["powell/nfev"] = np.array(int(res.nfev))
    meta["powell"] = dict(kind=kind, config=jsonable(cfg), init_policy=[25.0] * 4)
    print("powell policy=%s fun=%r nfev=%d" % (policy, float(res.fun), int(res.nfev)))
    out["meta"] = json.dumps(meta)
    np.savez_compressed(os.path.join(OUT, "base_stock.npz"), **out)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Golden vectors from the REFERENCE env classes on randomly drawn configurations.

The 30 hand-picked cases of tools/gen_fixtures.py all use the reference scripts' own constants
(capacity 30, delays 1-4, prices 5..1). This generator draws configurations across the space the
constructors accept: 2-8 serial stages or random trees (child index > parent, up to 3 children),
capacities from 5 to 40,000 (every state element width: uint8, int16 and int32 rows), initial
inventory, targets, prices and costs, delays 1-5, horizons 10-50, action bounds a < b, every
observation flag, standardised or raw state / actions, shared or independent rewards, noisy
delay with host-fed uniforms. Each case runs E envs through the reference with host-fed demand
and actions (the machinery and record format of tools/gen_fixtures.py), so the fixtures are data
only. Runs only in the build container (the reference is not on the GPU box).

    python tools/gen_fuzz_fixtures.py      # writes tests/golden/fuzz/*.npz, tests/golden/adaptor/fz_*.npz

Second part: drop-in adaptor sessions on drawn configurations with the reference's OWN randomness
(tools/gen_fixtures.py adaptor_script: constructor seed, scipy demand at reset, noisy demand and
noisy delay on NumPy's global stream), over Poisson / uniform / custom demand.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import gen_fixtures as gf  # noqa: E402
from fuzz_configs import fuzz_inputs, rand_config  # noqa: E402,F401

OUT = os.path.join(HERE, "..", "tests", "golden", "fuzz")
NUM_CASES = 24
E = 8


NUM_ADAPTOR = 12


def rand_adaptor_config(rs, kind, idx):
    """A drawn configuration (capacities up to 300) with the reference's own demand process."""
    cfg = rand_config(rs, kind, idx % 4)
    cfg.pop("demand_dist")
    tree = kind in ("IM_div", "MAIM_div")
    R = sum(1 for v in cfg["connections"].values() if not v) if tree else 1
    T = cfg["num_periods"]
    top = float(np.max(cfg["inv_max"]))
    dist = ["poisson", "uniform", "custom"][idx % 3]
    cfg["demand_dist"] = dist
    if dist == "poisson":
        cfg["mu"] = float(np.round(rs.uniform(0.05, 0.6) * top, 1))
    elif dist == "uniform":
        lo = int(rs.randint(0, max(2, int(top // 4))))
        cfg["lower_upper"] = (lo, lo + 1 + int(rs.randint(1, max(2, int(top // 2)))))
    else:
        shape = (R, T) if tree else (T,)
        cfg["customer_demand"] = rs.randint(0, max(2, int(top // 2)), size=shape)
    if tree and (idx // 4) % 2 == 0:       # cases 2, 3, 10, 11: custom, Poisson, uniform, custom demand
        cfg["noisy_demand"] = True
        cfg["noisy_demand_threshold"] = float(np.round(rs.uniform(0.05, 0.4), 2))
    if tree and idx >= 6:        # cases 6, 7, 10, 11; both div envs read noisy_delay from the config (IM_div_env.py:50-51)
        cfg["noisy_delay"] = True
        cfg["noisy_delay_threshold"] = float(np.round(rs.uniform(0.05, 0.4), 2))
    opts = {"noisy": float(np.round(rs.uniform(0.1, 0.5), 2))} if rs.rand() < 0.3 else {}
    return cfg, opts


def main():
    if not os.path.isdir(gf.REF):
        print("reference not mounted; nothing to do (fixtures are committed)")
        return
    classes = gf.import_reference()
    os.makedirs(OUT, exist_ok=True)
    gf.E = E
    gf.make_inputs = lambda kind, cfg, opts, seed: fuzz_inputs(kind, cfg, opts, seed, E)
    rs = np.random.RandomState(2024)
    kinds = ["IM", "MAIM", "IM_div", "MAIM_div"]
    for idx in range(NUM_CASES):
        kind = kinds[idx % 4]
        cfg = rand_config(rs, kind, idx)
        opts = {"noisy": float(np.round(rs.uniform(0.1, 0.5), 2))} if rs.rand() < 0.25 else {}
        gf.T = cfg["num_periods"]
        name = "fz%02d_%s" % (idx, kind)
        out = gf.run_case(classes, name, kind, cfg, opts, seed=5000 + idx)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
        print("%-16s N=%d T=%2d cap~%-6d flags td=%d pd=%d pa=%d L=%d noisy=%s errs=%d" % (
            name, cfg.get("num_stages", cfg.get("num_nodes")), cfg["num_periods"], int(np.max(cfg["inv_max"])),
            cfg["time_dependency"], cfg["prev_demand"], cfg["prev_actions"], cfg["prev_length"],
            opts.get("noisy", 0), int((out["err"] >= 0).sum())))
    # targeted: the flag combination the multi-agent classes have no observation branch for
    # (prev_demand alone: MAIM_env.py:296-317, MAIM_div_env.py:413-432), standardised, odd bounds
    for idx, kind in ((NUM_CASES, "MAIM"), (NUM_CASES + 1, "MAIM_div")):
        cfg = rand_config(rs, kind, idx)
        cfg.update(time_dependency=False, prev_demand=True, prev_actions=False, prev_length=2,
                   standardise_state=True, a=-2.0, b=1.0)
        if kind == "MAIM_div":
            cfg["share_network"] = True
        gf.T = cfg["num_periods"]
        name = "fz%02d_%s_pd_only" % (idx, kind)
        out = gf.run_case(classes, name, kind, cfg, {}, seed=5000 + idx)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
        print("%-16s (prev_demand alone)" % name)
    rs = np.random.RandomState(77)
    cases = {}
    for idx in range(NUM_ADAPTOR):
        kind = kinds[idx % 4]
        cfg, opts = rand_adaptor_config(rs, kind, idx)
        cases["fz_ad%02d_%s_%s" % (idx, kind, cfg["demand_dist"])] = (kind, cfg, opts)
    gf.ADAPTOR_CASES = cases
    gf.adaptor_traces(classes)


if __name__ == "__main__":
    main()

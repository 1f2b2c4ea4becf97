#!/usr/bin/env python3
"""Generate golden parity vectors by running the REFERENCE env classes.

Runs only in the build container, where the read-only reference is mounted at
/root/reference (it does not exist on the GPU box; the committed .npz files are
what travels). It imports environments/{IM_env,MAIM_env,IM_div_env,MAIM_div_env}.py
with tiny stand-ins for the two base classes it needs from packages that are
not installed here (gym.Env / gym.spaces.Box and ray.rllib.MultiAgentEnv carry no
arithmetic), steps every env with host-fed demand and actions, and records the
per-period history. Nothing from the reference is copied: the outputs are data.

    python tools/gen_fixtures.py            # writes tests/golden/*.npz, kat.json, adaptor/*.npz

Each case: E envs x T periods. Recorded (per period, after the step):
order, demand, acquisition, ship, inv, backlog, order_u, obs, reward, profit,
ship_to / backlog_to (trees), plus obs0 (reset obs) and err (step that raised).
"""
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def import_reference():
    sys.dont_write_bytecode = True   # keep the reference tree free of __pycache__
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")

    class Box:
        def __init__(self, low=None, high=None, shape=None, dtype=None):
            self.low, self.high, self.shape, self.dtype = low, high, shape, dtype

    class Env:
        pass

    spaces.Box = Box
    gym.spaces = spaces
    gym.Env = Env
    ray = types.ModuleType("ray")
    rllib = types.ModuleType("ray.rllib")

    class MultiAgentEnv:
        pass

    rllib.MultiAgentEnv = MultiAgentEnv
    ray.rllib = rllib
    agents = types.ModuleType("ray.rllib.agents")
    rllib.agents = agents
    sys.modules.update({"gym": gym, "gym.spaces": spaces, "ray": ray, "ray.rllib": rllib,
                        "ray.rllib.agents": agents})
    sys.path.insert(0, REF)
    from environments.IM_env import InvManagement
    from environments.MAIM_env import MultiAgentInvManagement
    from environments.IM_div_env import InvManagementDiv
    from environments.MAIM_div_env import MultiAgentInvManagementDiv
    return dict(IM=InvManagement, MAIM=MultiAgentInvManagement, IM_div=InvManagementDiv,
                MAIM_div=MultiAgentInvManagementDiv)


# ----------------------------------------------------------------- configs
def serial4(**kw):
    """inv_management.py:35-56 constants."""
    c = dict(num_stages=4, num_periods=30, init_inv=np.ones(4) * 10, inv_target=np.zeros(4),
             inv_max=np.ones(4) * 30, price=np.array([5, 4, 3, 2, 1]),
             stock_cost=np.array([0.35, 0.3, 0.4, 0.2]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.9]),
             delay=np.array([1, 2, 3, 1], dtype=np.int8), demand_dist="poisson", mu=5, seed=52,
             standardise_state=True, standardise_actions=True, a=-1, b=1,
             time_dependency=False, prev_demand=False, prev_actions=False, prev_length=1)
    c.update(kw)
    return c


def serial8(**kw):
    """SHLP_8.py:26-46 constants."""
    c = dict(num_stages=8, num_periods=30, init_inv=np.ones(8) * 10, inv_target=np.zeros(8),
             inv_max=np.ones(8) * 30, price=np.array([9, 8, 7, 6, 5, 4, 3, 2, 1]),
             stock_cost=np.array([0.35, 0.3, 0.4, 0.2, 0.35, 0.3, 0.4, 0.2]),
             backlog_cost=np.array([0.5, 0.7, 0.6, 0.9, 0.5, 0.7, 0.6, 0.9]),
             delay=np.array([1, 2, 3, 1, 4, 2, 3, 1], dtype=np.int8), demand_dist="poisson", mu=5,
             seed=52, standardise_state=True, standardise_actions=True, a=-1, b=1,
             time_dependency=False, prev_demand=False, prev_actions=False, prev_length=1)
    c.update(kw)
    return c


def div1(**kw):
    """MA_inv_management_div.py:46-69 constants."""
    c = dict(num_nodes=4, connections={0: [1], 1: [2, 3], 2: [], 3: []}, num_periods=30,
             init_inv=np.ones(4) * 10, inv_target=np.zeros(4), inv_max=np.ones(4) * 30,
             stock_cost=np.array([0.35, 0.3, 0.4, 0.4]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.6]),
             delay=np.array([1, 2, 1, 1], dtype=np.int8), demand_dist="poisson", mu=5, seed=52,
             time_dependency=False, prev_demand=False, prev_actions=False, prev_length=1,
             independent=False, share_network=False)
    c.update(kw)
    return c


def div2(**kw):
    """SHLP_div2.py / DSHLP_div2.py:21-40 topology (two split nodes)."""
    c = dict(num_nodes=6, connections={0: [1], 1: [2, 3], 2: [4, 5], 3: [], 4: [], 5: []},
             num_periods=30, init_inv=np.ones(6) * 10, inv_target=np.zeros(6), inv_max=np.ones(6) * 30,
             stock_cost=np.array([0.35, 0.3, 0.4, 0.4, 0.35, 0.3]),
             backlog_cost=np.array([0.5, 0.7, 0.6, 0.6, 0.5, 0.7]),
             delay=np.array([1, 2, 1, 1, 2, 1], dtype=np.int8), demand_dist="poisson", mu=5, seed=52,
             time_dependency=False, prev_demand=False, prev_actions=False, prev_length=1,
             independent=False, share_network=False)
    c.update(kw)
    return c


CASES = {
    # serial, single agent
    "C1_IM4": ("IM", serial4(), {}),
    "IM4_S3": ("IM", serial4(prev_demand=True, prev_actions=True), {}),
    "IM4_td_pd_pa_L2": ("IM", serial4(time_dependency=True, prev_demand=True, prev_actions=True, prev_length=2), {}),
    "IM4_pa_only": ("IM", serial4(prev_actions=True), {}),
    "IM4_nonstd": ("IM", serial4(standardise_state=False, standardise_actions=False), {"raw_actions": True}),
    "IM4_nonstd_td_pd": ("IM", serial4(standardise_state=False, time_dependency=True, prev_demand=True), {}),
    "IM4_noisy_delay": ("IM", serial4(time_dependency=True), {"noisy": 0.3}),
    "IM3_defaults": ("IM", dict(num_stages=3, num_periods=30, demand_dist="poisson", mu=5), {"mu_scale": 6}),
    "C3_IM8": ("IM", serial8(), {}),
    "IM8_td": ("IM", serial8(time_dependency=True, prev_demand=True), {}),
    # serial, multi agent
    "C2_MAIM4": ("MAIM", serial4(independent=False), {}),
    "MAIM4_indep": ("MAIM", serial4(independent=True), {}),
    "MAIM4_MA6": ("MAIM", serial4(independent=False, time_dependency=True, prev_demand=True), {}),
    "MAIM4_all_L2": ("MAIM", serial4(independent=False, time_dependency=True, prev_demand=True,
                                     prev_actions=True, prev_length=2), {}),
    "MAIM4_nonstd_td": ("MAIM", serial4(independent=False, standardise_state=False, time_dependency=True,
                                        prev_demand=True), {}),
    "MAIM4_nonstd_act": ("MAIM", serial4(independent=True, standardise_actions=False), {"raw_actions": True}),
    "MAIM4_noisy_delay": ("MAIM", serial4(independent=False, time_dependency=True), {"noisy": 0.3}),
    "MAIM3_defaults": ("MAIM", dict(num_stages=3, num_periods=30, demand_dist="poisson", mu=5), {"mu_scale": 6}),
    "MAIM8_td": ("MAIM", serial8(independent=False, time_dependency=True), {}),
    # tree, single agent
    "IM_div1": ("IM_div", div1(), {}),
    "IM_div1_td_pd_pa": ("IM_div", div1(time_dependency=True, prev_demand=True, prev_actions=True), {}),
    "IM_div1_nonstd": ("IM_div", div1(standardise_state=False, standardise_actions=False), {"raw_actions": True}),
    "IM_div1_noisy_delay": ("IM_div", div1(time_dependency=True), {"noisy": 0.3}),
    "IM_div2": ("IM_div", div2(time_dependency=True), {}),
    # tree, multi agent
    "C4_MAIM_div1": ("MAIM_div", div1(time_dependency=True, prev_demand=True), {}),
    "MAIM_div1_share": ("MAIM_div", div1(share_network=True, prev_demand=True, prev_actions=True), {}),
    "MAIM_div1_indep": ("MAIM_div", div1(independent=True, time_dependency=True), {}),
    "MAIM_div1_rev_children": ("MAIM_div", div1(connections={0: [1], 1: [3, 2], 2: [], 3: []},
                                                time_dependency=True), {}),
    "MAIM_div1_noisy_delay": ("MAIM_div", div1(time_dependency=True, prev_demand=True), {"noisy": 0.3}),
    "MAIM_div2_share": ("MAIM_div", div2(share_network=True, time_dependency=True, prev_demand=True,
                                         prev_actions=True, prev_length=2), {}),
}

E = 32          # envs per case
T = 30


def make_inputs(kind, cfg, opts, seed):
    rs = np.random.RandomState(seed)
    N = cfg.get("num_stages", cfg.get("num_nodes"))
    tree = kind in ("IM_div", "MAIM_div")
    if tree:
        conn = cfg["connections"]
        R = sum(1 for k, v in conn.items() if not v)
    else:
        R = 1
    mus = np.array([2, 5, 5, 10, 20, 40])[rs.randint(0, 6, size=E)] * opts.get("mu_scale", 1)
    dem = rs.poisson(mus[:, None, None], size=(E, R, T)).astype(np.int64)
    if opts.get("raw_actions"):
        om = 40.0
        act = rs.uniform(-5.0, om, size=(E, T, N))
        act[0] = 0.0
        act[1] = om
        act[2] = np.round(rs.uniform(0, 30, size=(T, N))) + 0.5    # exact .5 -> half-even rounding
    else:
        act = rs.uniform(-1.2, 1.2, size=(E, T, N))
        act[0] = 0.0
        act[1] = 1.0
        act[2] = -1.0
        act[3] = (rs.randint(0, 61, size=(T, N)) / 30.0) - 1.0     # grid incl. .5 round points
        act[4] = (rs.randint(0, 121, size=(T, N)) / 60.0) - 1.0
    unif = rs.uniform(0, 1, size=(E, T, N))
    return dem, act, unif


def run_case(classes, name, kind, cfg, opts, seed):
    Cls = classes[kind]
    N = cfg.get("num_stages", cfg.get("num_nodes"))
    tree = kind in ("IM_div", "MAIM_div")
    ma = kind in ("MAIM", "MAIM_div")
    dem, act, unif = make_inputs(kind, cfg, opts, seed)
    noisy = opts.get("noisy")
    rec = {k: [] for k in ("order", "demand", "acquisition", "ship", "inv", "backlog", "order_u", "obs",
                           "reward", "profit", "ship_to", "backlog_to")}
    obs0s, errs = [], []
    for e in range(E):
        env = Cls(dict(cfg))
        delay = np.asarray(env.delay)
        factory = 0 if tree else N - 1
        order_nodes = [factory] + [i for i in range(N) if i != factory]
        if tree:
            obs = env.reset(customer_demand=dem[e].copy(),
                            noisy_delay=bool(noisy), noisy_delay_threshold=noisy or 0)
        else:
            obs = env.reset(customer_demand=dem[e, 0].copy(),
                            noisy_delay=bool(noisy), noisy_delay_threshold=noisy or 0)
        obs0s.append(obs_array(obs, ma, N))
        per = {k: [] for k in rec}
        err = -1
        for t in range(T):
            # noisy delay: the env draws np.random.uniform per node (factory first, then the
            # others ascending) when t - delay >= 0; feed those draws from the per-(t,node) table.
            queue = [unif[e, t, i] for i in order_nodes if t - int(delay[i]) >= 0]
            orig = np.random.uniform
            np.random.uniform = lambda lo=0.0, hi=1.0, size=None, _q=queue: _q.pop(0)
            try:
                if ma:
                    names = ["node_%d" % i if tree else "stage_%d" % i for i in range(N)]
                    ad = {names[i]: np.array([act[e, t, i]]) for i in range(N)}
                    obs, r, done, info = env.step(ad)
                    rv = np.array([r[nm] for nm in names], dtype=np.float64)
                else:
                    obs, r, done, info = env.step(act[e, t].copy())
                    rv = np.array([r], dtype=np.float64)
            except Exception as ex:     # "Infinite Loop" guards
                err = t
                np.random.uniform = orig
                print("  %s env %d raised at t=%d: %s" % (name, e, t, ex))
                break
            finally:
                np.random.uniform = orig
            assert not (noisy and queue)
            per["order"].append(env.order_r[t].copy())
            per["demand"].append(env.demand[t].copy())
            per["acquisition"].append(env.acquisition[t].copy())
            per["ship"].append(env.ship[t].copy())
            per["inv"].append(env.inv[t + 1].copy())
            per["backlog"].append(env.backlog[t + 1].copy())
            per["order_u"].append(env.order_u[t + 1].copy())
            per["obs"].append(obs_array(obs, ma, N))
            per["reward"].append(rv)
            if ma:
                per["profit"].append(np.array([info[nm]["profit"] for nm in names]))
            else:
                per["profit"].append(np.asarray(info["profit"], dtype=np.float64))
            st = np.zeros(N)
            bt = np.zeros(N)
            if tree:
                for p, ch in env.connections.items():
                    for c in (ch or []):
                        st[c] = env.ship_to_list[t][p][c]
                for p, d in env.backlog_to.items():
                    for c, v in d.items():
                        bt[c] = v
            per["ship_to"].append(st)
            per["backlog_to"].append(bt)
        errs.append(err)
        for k in rec:
            arr = np.array(per[k], dtype=np.float64)
            full = np.full((T,) + (arr.shape[1:] if len(per[k]) else rec_shape(k, N, obs0s[-1], ma)), np.nan)
            full[:len(per[k])] = arr
            rec[k].append(full)
    out = {k: np.array(v) for k, v in rec.items()}
    out["obs0"] = np.array(obs0s)
    out["err"] = np.array(errs, dtype=np.int64)
    out["customer_demand"] = dem
    out["actions"] = act
    out["delay_uniforms"] = unif if noisy else np.zeros((0,))
    meta = dict(kind=kind, config=jsonable(cfg), noisy=noisy or 0.0, E=E, T=T, seed=seed)
    out["meta"] = np.array(json.dumps(meta))
    return out


def rec_shape(k, N, obs0, ma):
    if k == "obs":
        return obs0.shape
    if k == "reward":
        return (N,) if ma else (1,)
    return (N,)


def obs_array(obs, ma, N):
    if isinstance(obs, dict):
        keys = sorted(obs.keys(), key=lambda s: int(s.split("_")[1]))
        return np.array([obs[k] for k in keys], dtype=np.float64)
    return np.asarray(obs, dtype=np.float64)


def jsonable(cfg):
    out = {}
    for k, v in cfg.items():
        if isinstance(v, np.ndarray):
            out[k] = {"__nd__": v.tolist(), "dtype": str(v.dtype)}
        elif isinstance(v, dict):
            out[k] = {"__conn__": [[int(a), [int(c) for c in b]] for a, b in v.items()]}
        elif isinstance(v, (np.integer,)):
            out[k] = int(v)
        elif isinstance(v, (np.floating,)):
            out[k] = float(v)
        else:
            out[k] = v
    return out


def kats(classes):
    """KAT0-KAT3 of SURVEY.md §4, recomputed from the reference."""
    out = {}
    env = classes["IM"](serial4())
    out["KAT0_demand"] = [int(x) for x in env.customer_demand]
    R = 0.0
    for t in range(30):
        _, r, _, _ = env.step(np.zeros(4))
        R += r
    out["KAT1"] = dict(ret=float(R), inv=env.inv[30].tolist(), backlog=env.backlog[30].tolist(),
                       order_u=env.order_u[30].tolist(), demand=[int(x) for x in env.customer_demand])
    env = classes["MAIM"](serial4(independent=False))
    R = 0.0
    for t in range(30):
        _, r, _, _ = env.step({"stage_%d" % i: np.array([0.0]) for i in range(4)})
        R += sum(r.values())
    out["KAT2"] = dict(ret=float(R), demand=[int(x) for x in env.customer_demand])
    env = classes["MAIM_div"](div1(time_dependency=True, prev_demand=True))
    R = 0.0
    for t in range(30):
        obs, r, _, _ = env.step({"node_%d" % i: np.array([0.0]) for i in range(4)})
        R += sum(r.values())
    out["KAT3"] = dict(ret=float(R), backlog_to={str(k): {str(c): float(v) for c, v in d.items()}
                                                    for k, d in env.backlog_to.items()},
                       obs_node_1=[float(x) for x in obs["node_1"]],
                       demand=np.asarray(env.customer_demand).tolist())
    return out


# ----------------------------------------------------------------- adaptor traces
# Scripted sessions with the reference's OWN randomness (np.random.seed in the constructor, scipy
# demand draws at reset, noisy-delay / noisy-demand uniforms on the global stream): construct,
# run the constructor's episode, reset, run 10 steps, reset mid-episode (optionally latching noisy
# delay), run a full episode. Actions come from a separate RandomState so the global stream is the
# env's alone. tests/test_adaptors_gpu.py replays the same script on imenv.envs.
ADAPTOR_CASES = {
    "ad_IM4_mu3": ("IM", serial4(mu=3), {}),
    "ad_IM4_custom": ("IM", serial4(demand_dist="custom", customer_demand=np.arange(30) % 7), {}),
    "ad_IM4_noisy": ("IM", serial4(time_dependency=True), {"noisy": 0.3}),
    "ad_MAIM4_mu3": ("MAIM", serial4(independent=False, mu=3), {}),
    "ad_MAIM4_uniform_indep_noisy": ("MAIM", serial4(independent=True, demand_dist="uniform",
                                                     lower_upper=(2, 7), time_dependency=True), {"noisy": 0.4}),
    "ad_IM_div1_noisy_demand": ("IM_div", div1(noisy_demand=True, noisy_demand_threshold=0.2,
                                               time_dependency=True), {}),
    "ad_MAIM_div1_cfg_noisy_delay": ("MAIM_div", div1(time_dependency=True, prev_demand=True, noisy_delay=True,
                                                      noisy_delay_threshold=0.25), {}),
    "ad_MAIM_div2_share": ("MAIM_div", div2(share_network=True, time_dependency=True), {}),
}


def adaptor_script(env, kind, opts, rs, record):
    """The session both the reference and the adaptor run (tests/test_adaptors_gpu.py)."""
    ma = kind in ("MAIM", "MAIM_div")
    prefix = "stage_" if kind == "MAIM" else "node_"
    N = env.num_nodes if hasattr(env, "num_nodes") else env.num_stages
    T = env.num_periods
    record("reset", env.state, env.customer_demand)

    def run(steps):
        for _ in range(steps):
            x = rs.uniform(-1.05, 1.05, size=N)
            act = {prefix + str(i): np.array([x[i]]) for i in range(N)} if ma else x
            out = env.step(act)
            record("step", *out)

    run(T)
    record("reset", env.reset(), env.customer_demand)
    run(10)
    if "noisy" in opts:
        record("reset", env.reset(noisy_delay=True, noisy_delay_threshold=opts["noisy"]), env.customer_demand)
    else:
        record("reset", env.reset(), env.customer_demand)
    run(T)


def adaptor_traces(classes):
    for name, (kind, cfg, opts) in ADAPTOR_CASES.items():
        ma = kind in ("MAIM", "MAIM_div")
        meta_cfg = jsonable(cfg)    # before the session: the reference mutates a custom demand array in place
        caller = dict(cfg)
        env = classes[kind](caller)
        rec = {"reset_obs": [], "reset_demand": [], "obs": [], "reward": [], "done": [], "period": [],
               "demand": [], "ship": [], "acquisition": [], "profit": [], "actual_order": []}
        N = env.num_nodes if hasattr(env, "num_nodes") else env.num_stages

        def record(what, *args):
            if what == "reset":
                rec["reset_obs"].append(obs_array(args[0], ma, N))
                rec["reset_demand"].append(np.array(args[1], dtype=np.int64).reshape(-1))   # a copy
                return
            obs, r, d, info = args
            rec["obs"].append(obs_array(obs, ma, N))
            if ma:
                keys = sorted(r.keys(), key=lambda s: int(s.split("_")[1]))
                rec["reward"].append(np.array([r[k] for k in keys], dtype=np.float64))
                rec["done"].append(bool(d["__all__"]))
                ik = sorted(info.keys(), key=lambda s: int(s.split("_")[1]))
                rec["period"].append(info[ik[0]]["period"])
                for f, src in (("demand", "demand"), ("ship", "ship"), ("acquisition", "acquisition"),
                               ("profit", "profit"), ("actual_order", "actual order")):
                    rec[f].append(np.array([info[k][src] for k in ik], dtype=np.float64))
            else:
                rec["reward"].append(np.array([r], dtype=np.float64))
                rec["done"].append(bool(d))
                rec["period"].append(info["period"])
                for f in ("demand", "ship", "acquisition", "profit"):
                    rec[f].append(np.asarray(info[f], dtype=np.float64).copy())
                rec["actual_order"].append(np.zeros(N))

        adaptor_script(env, kind, opts, np.random.RandomState(7), record)
        out = {k: np.array(v) for k, v in rec.items() if k != "reset_demand"}
        out["reset_demand"] = np.array(rec["reset_demand"])
        out["meta"] = json.dumps(dict(kind=kind, config=meta_cfg, opts=opts,
                                      caller_keys_after=sorted(caller.keys())))
        os.makedirs(os.path.join(OUT, "adaptor"), exist_ok=True)
        np.savez_compressed(os.path.join(OUT, "adaptor", name + ".npz"), **out)
        print("%-30s %-9s steps=%d" % (name, kind, len(rec["obs"])))


def main():
    if not os.path.isdir(REF):
        print("reference not mounted; nothing to do (fixtures are committed)")
        return
    classes = import_reference()
    os.makedirs(OUT, exist_ok=True)
    for idx, (name, (kind, cfg, opts)) in enumerate(CASES.items()):
        out = run_case(classes, name, kind, cfg, opts, seed=1000 + idx)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
        print("%-26s %-9s errs=%d" % (name, kind, int((out["err"] >= 0).sum())))
    with open(os.path.join(OUT, "kat.json"), "w") as f:
        json.dump(kats(classes), f, indent=1)
    adaptor_traces(classes)


if __name__ == "__main__":
    main()

"""Drop-in adaptors (imenv.envs) vs the reference's own seeded sessions.

tests/golden/adaptor/*.npz were recorded by tools/gen_fixtures.py running the reference classes with
their own randomness (np.random.seed in the constructor, scipy demand draws, noisy-demand and
noisy-delay uniforms on NumPy's global stream). The adaptor replays the same script; everything it
returns must be identical: reset observations and drawn demand, per-step observations, rewards,
done flags and the info values, plus the keys the constructor leaves in the caller's config dict.
"""
import json

import numpy as np
import pytest

from golden_io import adaptor_case_names, decode_config, load_adaptor_case, load_kat

pytestmark = pytest.mark.gpu


def _classes():
    from imenv import envs
    return dict(IM=envs.InvManagement, MAIM=envs.MultiAgentInvManagement, IM_div=envs.InvManagementDiv,
                MAIM_div=envs.MultiAgentInvManagementDiv)


def _obs_array(obs, ma):
    if ma:
        keys = sorted(obs.keys(), key=lambda s: int(s.split("_")[1]))
        return np.array([obs[k] for k in keys], dtype=np.float64)
    return np.asarray(obs, dtype=np.float64)


def _script(env, kind, opts, rs, record):
    """Same session as tools/gen_fixtures.py:adaptor_script."""
    ma = kind in ("MAIM", "MAIM_div")
    prefix = "stage_" if kind == "MAIM" else "node_"
    N, T = env.num_nodes, env.num_periods
    record("reset", env.state, env.customer_demand)

    def run(steps):
        for _ in range(steps):
            x = rs.uniform(-1.05, 1.05, size=N)
            act = {prefix + str(i): np.array([x[i]]) for i in range(N)} if ma else x
            record("step", *env.step(act))

    run(T)
    record("reset", env.reset(), env.customer_demand)
    run(10)
    if "noisy" in opts:
        record("reset", env.reset(noisy_delay=True, noisy_delay_threshold=opts["noisy"]), env.customer_demand)
    else:
        record("reset", env.reset(), env.customer_demand)
    run(T)


@pytest.mark.parametrize("name", adaptor_case_names())
def test_adaptor_reproduces_reference_session(name):
    meta, ref = load_adaptor_case(name)
    kind = meta["kind"]
    ma = kind in ("MAIM", "MAIM_div")
    caller = decode_config(meta["config"])
    env = _classes()[kind](caller)
    assert sorted(caller.keys()) == meta["caller_keys_after"]
    got = {k: [] for k in ("reset_obs", "reset_demand", "obs", "reward", "done", "period", "demand", "ship",
                           "acquisition", "profit", "actual_order")}

    def record(what, *args):
        if what == "reset":
            got["reset_obs"].append(_obs_array(args[0], ma))
            got["reset_demand"].append(np.array(args[1], dtype=np.int64).reshape(-1))   # a copy
            return
        obs, r, d, info = args
        got["obs"].append(_obs_array(obs, ma))
        if ma:
            keys = sorted(r.keys(), key=lambda s: int(s.split("_")[1]))
            got["reward"].append(np.array([r[k] for k in keys]))
            got["done"].append(bool(d["__all__"]))
            ik = sorted(info.keys(), key=lambda s: int(s.split("_")[1]))
            got["period"].append(info[ik[0]]["period"])
            for f, src in (("demand", "demand"), ("ship", "ship"), ("acquisition", "acquisition"),
                           ("profit", "profit"), ("actual_order", "actual order")):
                got[f].append(np.array([info[k][src] for k in ik], dtype=np.float64))
        else:
            got["reward"].append(np.array([r], dtype=np.float64))
            got["done"].append(bool(d))
            got["period"].append(info["period"])
            for f in ("demand", "ship", "acquisition", "profit"):
                got[f].append(np.asarray(info[f], dtype=np.float64).copy())
            got["actual_order"].append(np.zeros(env.num_nodes))

    _script(env, kind, meta["opts"], np.random.RandomState(7), record)
    for k, v in got.items():
        np.testing.assert_array_equal(np.array(v), ref[k], err_msg="%s/%s" % (name, k))
    env.close()


def test_adaptor_known_answers():
    """KAT1-KAT3: zero actions from the constructor's own episode."""
    from imenv import envs
    kat = load_kat()
    cfg4 = dict(num_stages=4, num_periods=30, init_inv=np.ones(4) * 10, inv_target=np.zeros(4),
                inv_max=np.ones(4) * 30, price=np.array([5, 4, 3, 2, 1]),
                stock_cost=np.array([0.35, 0.3, 0.4, 0.2]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.9]),
                delay=np.array([1, 2, 3, 1], dtype=np.int8), demand_dist="poisson", mu=5, seed=52,
                standardise_state=True, standardise_actions=True, a=-1, b=1,
                time_dependency=False, prev_demand=False, prev_actions=False, prev_length=1)
    env = envs.InvManagement(dict(cfg4))
    assert [int(x) for x in env.customer_demand] == kat["KAT0_demand"]
    R = 0.0
    for _ in range(30):
        _, r, _, _ = env.step(np.zeros(4))
        R += r
    assert R == kat["KAT1"]["ret"]
    assert env.inv[30].tolist() == kat["KAT1"]["inv"]
    assert env.backlog[30].tolist() == kat["KAT1"]["backlog"]
    assert env.order_u[30].tolist() == kat["KAT1"]["order_u"]
    env = envs.MultiAgentInvManagement(dict(cfg4, independent=False))
    R = 0.0
    for _ in range(30):
        _, r, _, _ = env.step({"stage_%d" % i: np.array([0.0]) for i in range(4)})
        R += sum(r.values())
    assert R == kat["KAT2"]["ret"]
    div = dict(num_nodes=4, connections={0: [1], 1: [2, 3], 2: [], 3: []}, num_periods=30,
               init_inv=np.ones(4) * 10, inv_target=np.zeros(4), inv_max=np.ones(4) * 30,
               stock_cost=np.array([0.35, 0.3, 0.4, 0.4]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.6]),
               delay=np.array([1, 2, 1, 1], dtype=np.int8), demand_dist="poisson", mu=5, seed=52,
               time_dependency=True, prev_demand=True, prev_actions=False, prev_length=1,
               independent=False, share_network=False)
    env = envs.MultiAgentInvManagementDiv(div)
    R = 0.0
    for _ in range(30):
        obs, r, _, _ = env.step({"node_%d" % i: np.array([0.0]) for i in range(4)})
        R += sum(r.values())
    assert R == kat["KAT3"]["ret"]
    assert [float(x) for x in obs["node_1"]] == kat["KAT3"]["obs_node_1"]


def test_adaptor_step_past_horizon_raises():
    from imenv import envs
    env = envs.InvManagement(dict(num_stages=3, num_periods=5, demand_dist="poisson", mu=5))
    for _ in range(5):
        env.step(np.zeros(3))
    with pytest.raises(IndexError):
        env.step(np.zeros(3))

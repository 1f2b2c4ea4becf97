"""Fused base-stock rollout (imenv_base_stock_rollout / imenv.policy) vs the reference and the oracle.

* Golden: tests/golden/base_stock.npz holds what the reference's base_restock_policy.py computes
  (dfo_func objectives, evaluation-loop returns, state sums) for P policies x S demand rows of
  seven configurations (serial 4/8 stages, standardised actions, uniform demand, two trees). The
  GPU must reproduce every per-episode value bit for bit.
* Drop-in: imenv.policy.dfo_func on the adaptor env returns the reference's objective, and
  optimize_inventory_policy retraces the reference's Powell search (same nfev, x, fun, policy).
* In-kernel demand (Philox) and noisy delay vs oracle/base_stock.py with the same keys.
* Sizes: P x S up to 8 x 20,000 episodes vs the oracle; policy_stats vs np.mean / np.std.
"""
import numpy as np
import pytest
import torch

from golden_io import load_base_stock
from oracle import base_stock as bs

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
META, CASES = load_base_stock()
ROLL = [c for c in CASES if c != "powell"]
STATS = ("return", "objective", "inventory", "backlog", "customer_backlog")


def _rollout(kind, cfg):
    from imenv.policy import BaseStockRollout
    return BaseStockRollout(kind, cfg, device=DEV)


def _pmf(cfg):
    from scipy.stats import poisson, randint
    if cfg.get("demand_dist") == "uniform":
        lo, hi = cfg["lower_upper"]
        return lambda k: randint.pmf(k, low=lo, high=hi)
    return lambda k: poisson.pmf(k, mu=cfg.get("mu", 5))


@pytest.mark.parametrize("name", ROLL)
def test_rollout_matches_reference_golden(name):
    m, d = META[name], CASES[name]
    ro = _rollout(m["kind"], m["config"])
    out = ro.run(d["policies"], demand=d["demand"])
    for k in STATS:
        np.testing.assert_array_equal(out[k].cpu().numpy(), d[k], err_msg="%s %s" % (name, k))
    st = out["stats"].cpu().numpy()
    for j, k in enumerate(STATS):
        np.testing.assert_allclose(st[:, j, 0], np.mean(d[k], axis=1), rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(st[:, j, 1], np.std(d[k], axis=1), rtol=1e-9, atol=1e-12)
    assert "rollout jit:imenv_rollout_jit" in ro.kernel_info()
    ro.close()


def _retailers(cfg):
    return sum(1 for v in cfg["connections"].values() if not v)


@pytest.mark.parametrize("name", [c for c in ROLL if META[c]["kind"] in ("IM_div", "MAIM_div")
                                  and _retailers(META[c]["config"]) > 1])
@pytest.mark.parametrize("replay", ["0", "1"])
def test_tree_objective_single_pass_and_replay(name, replay, monkeypatch):
    """Trees (R > 1 retailer rows): the single-pass kernel parks rows 1..R-1 of the objective's terms
    (tb > 0) and the replay kernel re-runs the episode per row (IMENV_ROLLOUT_REPLAY=1, tb=0); both
    give the reference's np.sum order bit for bit."""
    monkeypatch.setenv("IMENV_ROLLOUT_REPLAY", replay)
    m, d = META[name], CASES[name]
    ro = _rollout(m["kind"], m["config"])
    out = ro.run(d["policies"], demand=d["demand"])
    for k in STATS:
        np.testing.assert_array_equal(out[k].cpu().numpy(), d[k], err_msg="%s %s" % (name, k))
    assert (",tb=0," in ro.kernel_info()) == (replay == "1"), ro.kernel_info()
    ro.close()


def test_dfo_func_and_powell_drop_in():
    """imenv.policy.dfo_func / optimize_inventory_policy on the InvManagement adaptor reproduce the
    reference's objective and its whole Powell search (inv_management.py:217-218)."""
    from imenv import envs
    from imenv.policy import dfo_func, optimize_inventory_policy
    m, d = META["IM4_dfo"], CASES["IM4_dfo"]
    env = envs.InvManagement(dict(m["config"]), device=DEV)
    for p in range(d["policies"].shape[0]):
        for s in range(3):
            assert dfo_func(d["policies"][p], env, d["demand"][s]) == d["objective"][p, s]
    pw = CASES["powell"]
    policy, res = optimize_inventory_policy(env, dfo_func, init_policy=np.ones(4) * 25, demand=pw["demand"])
    assert res.nfev == int(pw["nfev"])
    np.testing.assert_array_equal(res.x, pw["x"])
    assert res.fun == float(pw["fun"])
    np.testing.assert_array_equal(policy, pw["policy"])


def test_evaluate_base_stock_matches_reference_loop():
    from imenv import envs
    from imenv.policy import evaluate_base_stock
    m, d = META["IM4_dfo"], CASES["IM4_dfo"]
    env = envs.InvManagement(dict(m["config"]), device=DEV)
    r = evaluate_base_stock(env, d["policies"][1], d["demand"])
    np.testing.assert_array_equal(r, d["return"][1])


@pytest.mark.parametrize("case", [
    ("IM", "serial4", dict(), 0.0),
    ("IM", "serial4", dict(), 0.3),
    ("MAIM", "serial4", dict(independent=False), 0.2),
    ("IM", "serial8", dict(), 0.25),
    ("IM_div", "div1", dict(noisy_demand=True, noisy_demand_threshold=0.3), 0.3),
    ("IM", "serial4", dict(demand_dist="uniform", lower_upper=(2, 9)), 0.0),
])
def test_rollout_drawn_demand_and_noisy_delay_vs_oracle(case):
    """In-kernel Philox demand (+ noisy demand) and noisy delay: the same keyed draws as the oracle
    twin, so every per-episode metric is bit-exact (objective included)."""
    import gen_cfg
    kind, base, kw, thr = case
    cfg = getattr(gen_cfg, base)(standardise_state=False, standardise_actions=False, **kw)
    P, S, off, ep = 3, 700, 5000, 4
    rs = np.random.RandomState(1)
    N = cfg.get("num_stages", cfg.get("num_nodes"))
    pol = rs.uniform(0, 50, size=(P, N))
    ro = _rollout(kind, cfg)
    out = ro.run(pol, n_scenarios=S, scenario_offset=off, episode=ep, noisy_delay=thr > 0,
                 noisy_delay_threshold=thr)
    dist = cfg.get("demand_dist", "poisson")
    rng = dict(seed=cfg["seed"], episode=ep, env_offset=off, dist=dist, mu=cfg.get("mu", 5),
               lower_upper=cfg.get("lower_upper", (1, 5)))
    ref = bs.rollout(kind, cfg, pol, n_scenarios=S, rng=rng, pmf=_pmf(cfg), noisy_delay=thr > 0,
                     noisy_delay_threshold=thr)
    for k in STATS:
        np.testing.assert_array_equal(out[k].cpu().numpy(), ref[k], err_msg=k)
    ro.close()


def test_rollout_large_batch_stats():
    """8 policies x 20,000 drawn scenarios (~4.8 M env-steps): per-episode values bit-exact vs the
    oracle, policy_stats within 1e-12 of np.mean / np.std; S is not a multiple of the block."""
    import gen_cfg
    cfg = gen_cfg.serial4(standardise_state=False, standardise_actions=False)
    P, S = 8, 20000
    pol = np.stack([np.ones(4) * v for v in (5, 10, 15, 20, 25, 30, 40, 60)])
    ro = _rollout("IM", cfg)
    out = ro.run(pol, n_scenarios=S, episode=11)
    rng = dict(seed=cfg["seed"], episode=11, env_offset=0, dist="poisson", mu=5)
    ref = bs.rollout("IM", cfg, pol, n_scenarios=S, rng=rng, pmf=_pmf(cfg))
    for k in STATS:
        np.testing.assert_array_equal(out[k].cpu().numpy(), ref[k], err_msg=k)
    st = out["stats"].cpu().numpy()
    ref_st = bs.policy_stats(ref)
    np.testing.assert_allclose(st, ref_st, rtol=1e-12, atol=1e-9)
    # without per-episode outputs the kernel still produces the same stats (internal scratch)
    st2 = ro.run(pol, n_scenarios=S, episode=11, per_episode=False)["stats"].cpu().numpy()
    np.testing.assert_array_equal(st, st2)
    ro.close()


def test_rollout_errors():
    import gen_cfg
    from imenv import ImEnvNativeError
    ro = _rollout("MAIM", gen_cfg.serial4(independent=True))
    with pytest.raises(ImEnvNativeError, match="scalar reward"):
        ro.run(np.ones((1, 4)) * 10, n_scenarios=4)
    ro.close()
    ro = _rollout("IM", gen_cfg.serial4())
    with pytest.raises(ValueError):
        ro.run(np.array([[np.nan, 1, 1, 1]]), n_scenarios=4)
    with pytest.raises(ValueError):
        ro.run(np.ones((1, 3)), n_scenarios=4)
    ro.close()


@pytest.mark.parametrize("i", range(8))
def test_rollout_drawn_configs_vs_oracle(i):
    """The fused rollout on drawn single-agent configurations (tests/fuzz_configs.py: IM and IM_div,
    capacities 5-450, explicit order_max, raw or standardised actions), in-kernel Poisson or uniform
    demand, noisy demand on trees, noisy delay: every per-episode metric equals the oracle."""
    from fuzz_configs import maybe_order_max, rand_config
    rs = np.random.RandomState(4242 + i)
    kind = ("IM", "IM_div")[i % 2]
    while True:
        cfg = maybe_order_max(rs, kind, rand_config(rs, kind, (i // 2) % 4))
        R = sum(1 for v in cfg["connections"].values() if not v) if kind == "IM_div" else 1
        if R * cfg["num_periods"] <= 128:       # the objective's pairwise-sum block
            break
    top = float(np.max(cfg["inv_max"]))
    if i % 3 == 2:
        lo = int(rs.randint(0, max(2, int(top // 4))))
        cfg.update(demand_dist="uniform", lower_upper=(lo, lo + 2 + int(rs.randint(0, max(2, int(top // 2))))))
    else:
        cfg.update(demand_dist="poisson", mu=float(np.round(rs.uniform(0.05, 0.5) * top, 1)))
    if kind == "IM_div" and rs.rand() < 0.5:
        cfg.update(noisy_demand=True, noisy_demand_threshold=0.25)
    thr = 0.3 if rs.rand() < 0.5 else 0.0
    N = cfg.get("num_stages", cfg.get("num_nodes"))
    P, S, off, ep = 3, 300, int(rs.randint(0, 1 << 20)), int(rs.randint(0, 50))
    pol = rs.uniform(0, 1.5 * top, size=(P, N))
    ro = _rollout(kind, cfg)
    out = ro.run(pol, n_scenarios=S, scenario_offset=off, episode=ep, noisy_delay=thr > 0,
                 noisy_delay_threshold=thr)
    rng = dict(seed=cfg["seed"], episode=ep, env_offset=off, dist=cfg["demand_dist"], mu=cfg.get("mu", 5),
               lower_upper=cfg.get("lower_upper", (1, 5)))
    ref = bs.rollout(kind, cfg, pol, n_scenarios=S, rng=rng, pmf=_pmf(cfg), noisy_delay=thr > 0,
                     noisy_delay_threshold=thr)
    for k in STATS:
        np.testing.assert_array_equal(out[k].cpu().numpy(), ref[k], err_msg="%d %s" % (i, k))
    ro.close()

"""Fused plan replay (imenv_plan_rollout / imenv.plan) vs the reference and the oracle.

* Golden: tests/golden/plan_replay.npz holds what the LP scripts' evaluation loop computes on the
  reference env classes (SHLP_8.py:737-766: lp_reward, the observation sums, profit[j, t]) for LP-like
  plans on serial 4/8-stage chains, both trees and drawn configurations, with per-scenario and shared
  plans. The GPU reproduces every per-episode value and per-step reward bit for bit, from float64
  plans; float32 plans equal the oracle replaying the same float32 values.
* In-kernel demand (Philox), noisy demand and noisy delay vs oracle/plan.py with the same keys.
* Sizes up to 4 plans x 20,000 scenarios; policy_stats vs np.mean / np.std.
"""
import numpy as np
import pytest
import torch

from golden_io import load_base_stock
from oracle import plan as pl

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
META, CASES = load_base_stock("plan_replay.npz")
STATS = ("return", "inventory", "backlog", "customer_backlog")


def _pr(kind, cfg):
    from imenv.plan import PlanRollout
    return PlanRollout(kind, cfg, device=DEV)


def _kernel_plans(d, layout):
    """fixture plans ([T, P, S, N] per episode / [P, T, N] shared) -> PlanRollout's input layout."""
    return np.transpose(d["plans"], (1, 2, 0, 3)) if layout == "episode" else d["plans"]


@pytest.mark.parametrize("name", sorted(CASES))
def test_plan_replay_matches_reference_golden(name):
    m, d = META[name], CASES[name]
    pr = _pr(m["kind"], m["config"])
    out = pr.run(_kernel_plans(d, m["layout"]), demand=d["demand"], per_episode=m["layout"] == "episode")
    for k in STATS:
        np.testing.assert_array_equal(out[k].cpu().numpy(), d[k], err_msg="%s %s" % (name, k))
    np.testing.assert_array_equal(out["rewards"].cpu().numpy(), np.transpose(d["rewards"], (1, 2, 0)))
    st = out["stats"].cpu().numpy()
    for k in STATS:
        j = ("return", "objective", "inventory", "backlog", "customer_backlog").index(k)
        np.testing.assert_allclose(st[:, j, 0], np.mean(d[k], axis=1), rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(st[:, j, 1], np.std(d[k], axis=1), rtol=1e-9, atol=1e-12)
    assert "rollout jit:imenv_rollout_jit" in pr.kernel_info()
    pr.close()


def test_replay_plans_drop_in_lists():
    """replay_plans returns the LP scripts' lists (lp_reward_list, ...) and profit[j, t] for one
    per-scenario plan set: the SHLP_8 case of the fixtures."""
    from imenv import build_spec
    from imenv.plan import replay_plans
    m, d = META["SHLP8"], CASES["SHLP8"]
    res = replay_plans(build_spec(m["kind"], m["config"]), d["plans"][:, 0].transpose(1, 0, 2), d["demand"],
                       device=DEV)
    np.testing.assert_array_equal(res["lp_reward_list"], d["return"][0])
    np.testing.assert_array_equal(res["inventory_list"], d["inventory"][0])
    np.testing.assert_array_equal(res["backlog_list"], d["backlog"][0])
    np.testing.assert_array_equal(res["customer_backlog_list"], d["customer_backlog"][0])
    np.testing.assert_array_equal(res["profit"], d["rewards"][:, 0].T)


@pytest.mark.parametrize("name", ["SHLP4", "div1_shared"])
def test_plan_replay_f32_plans_vs_oracle(name):
    """float32 plans promote exactly to float64 (as step() does): equal to the oracle on the same values."""
    m, d = META[name], CASES[name]
    plans32 = _kernel_plans(d, m["layout"]).astype(np.float32)
    pr = _pr(m["kind"], m["config"])
    out = pr.run(torch.as_tensor(plans32), demand=d["demand"], per_episode=m["layout"] == "episode")
    ref_plans = np.transpose(plans32, (2, 0, 1, 3)) if m["layout"] == "episode" else plans32
    ref = pl.plan_rollout(m["kind"], m["config"], ref_plans.astype(np.float64),
                          per_episode=m["layout"] == "episode", demand=d["demand"])
    for k in STATS:
        np.testing.assert_array_equal(out[k].cpu().numpy(), ref[k], err_msg=k)
    np.testing.assert_array_equal(out["rewards"].cpu().numpy(), np.transpose(ref["rewards"], (1, 2, 0)))
    pr.close()


@pytest.mark.parametrize("case", [
    ("IM", "serial4", dict(), 0.0, "episode"),
    ("IM", "serial4", dict(), 0.3, "shared"),
    ("MAIM", "serial4", dict(independent=False), 0.2, "episode"),
    ("IM", "serial8", dict(), 0.25, "episode"),
    ("IM_div", "div1", dict(noisy_demand=True, noisy_demand_threshold=0.3), 0.3, "shared"),
    ("IM_div", "div2", dict(), 0.0, "episode"),
    ("IM", "serial4", dict(demand_dist="uniform", lower_upper=(2, 9)), 0.0, "episode"),
])
def test_plan_replay_drawn_demand_and_noisy_delay_vs_oracle(case):
    """In-kernel Philox demand (+ noisy demand) and noisy delay: the oracle's keyed twin draws, every
    per-episode metric and per-step reward bit-exact. Multi-agent shared rewards included."""
    import gen_cfg
    kind, base, kw, thr, layout = case
    cfg = getattr(gen_cfg, base)(standardise_state=False, standardise_actions=False, **kw)
    P, S, off, ep = 2, 500, 7000, 3
    rs = np.random.RandomState(7)
    N = cfg.get("num_stages", cfg.get("num_nodes"))
    T = cfg.get("num_periods", 30)
    plans = rs.randint(0, 25, size=(P, S, T, N) if layout == "episode" else (P, T, N)).astype(np.float64)
    plans += rs.choice([0.0, 0.5, -0.5, 1e-9], size=plans.shape)
    pr = _pr(kind, cfg)
    out = pr.run(plans, n_scenarios=S, scenario_offset=off, episode=ep, per_episode=layout == "episode",
                 noisy_delay=thr > 0, noisy_delay_threshold=thr)
    rng = dict(seed=cfg["seed"], episode=ep, env_offset=off, dist=cfg.get("demand_dist", "poisson"),
               mu=cfg.get("mu", 5), lower_upper=cfg.get("lower_upper", (1, 5)))
    ref_plans = np.transpose(plans, (2, 0, 1, 3)) if layout == "episode" else plans
    ref = pl.plan_rollout(kind, cfg, ref_plans, per_episode=layout == "episode", n_scenarios=S, rng=rng,
                          noisy_delay=thr > 0, noisy_delay_threshold=thr)
    for k in STATS:
        np.testing.assert_array_equal(out[k].cpu().numpy(), ref[k], err_msg=k)
    np.testing.assert_array_equal(out["rewards"].cpu().numpy(), np.transpose(ref["rewards"], (1, 2, 0)))
    pr.close()


def test_plan_replay_large_batch_stats():
    """4 shared plans x 20,000 drawn scenarios (2.4 M env-steps), S not a multiple of the block:
    per-episode values bit-exact vs the oracle, policy_stats within 1e-12 of np.mean / np.std,
    and the same stats without per-episode outputs or per-step rewards."""
    import gen_cfg
    from oracle.base_stock import policy_stats
    cfg = gen_cfg.serial4(standardise_state=False, standardise_actions=False)
    P, S, T = 4, 20000, 30
    rs = np.random.RandomState(3)
    plans = rs.randint(0, 15, size=(P, T, 4)).astype(np.float64)
    pr = _pr("IM", cfg)
    out = pr.run(plans, n_scenarios=S, episode=2)
    rng = dict(seed=cfg["seed"], episode=2, env_offset=0, dist="poisson", mu=5)
    ref = pl.plan_rollout("IM", cfg, plans, n_scenarios=S, rng=rng)
    for k in STATS:
        np.testing.assert_array_equal(out[k].cpu().numpy(), ref[k], err_msg=k)
    st = out["stats"].cpu().numpy()
    np.testing.assert_allclose(st, policy_stats(ref), rtol=1e-12, atol=1e-9)
    st2 = pr.run(plans, n_scenarios=S, episode=2, rewards=False, per_episode_stats=False)["stats"].cpu().numpy()
    np.testing.assert_array_equal(st, st2)
    pr.close()


def test_plan_replay_errors():
    import gen_cfg
    from imenv import ImEnvNativeError
    pr = _pr("MAIM", gen_cfg.serial4(independent=True))
    with pytest.raises(ImEnvNativeError, match="scalar reward"):
        pr.run(np.ones((30, 4)), n_scenarios=4)
    pr.close()
    # raw-state sums only: a standardised-state spec (the LP scripts never use one) is refused
    pr = _pr("IM", gen_cfg.serial4(standardise_state=True))
    with pytest.raises(ImEnvNativeError, match="standardise_state"):
        pr.run(np.ones((30, 4)), n_scenarios=4)
    pr.close()
    pr = _pr("MAIM_div", gen_cfg.div1(independent=False))
    with pytest.raises(ImEnvNativeError, match="standardise_state"):
        pr.run(np.ones((30, 4)), n_scenarios=4)
    pr.close()
    pr = _pr("IM", gen_cfg.serial4(standardise_state=False))
    with pytest.raises(ValueError):
        pr.run(np.ones((30, 3)), n_scenarios=4)                     # wrong node count
    with pytest.raises(ValueError):
        pr.run(np.ones((4, 29, 4)), per_episode=True)                # too few periods
    with pytest.raises(ValueError):
        pr.run(np.ones((30, 4)))                                     # shared plan, no scenario count
    pr.close()


def test_plan_replay_sharded_scenarios_equal_one_launch():
    """Scenarios split across two launches (scenario_offset = a rank's first global scenario id, as
    imenv.shard assigns them) give the same per-episode values and rewards as one launch over all of
    them: the in-kernel draws are keyed by global scenario id."""
    import gen_cfg
    cfg = gen_cfg.div1(standardise_state=False, standardise_actions=False, noisy_demand=True,
                       noisy_demand_threshold=0.2)
    S, T, N, half = 1000, 30, 4, 400
    rs = np.random.RandomState(11)
    plans = rs.randint(0, 20, size=(1, S, T, N)).astype(np.float64)
    pr = _pr("IM_div", cfg)
    whole = pr.run(plans, per_episode=True, n_scenarios=S, episode=5, noisy_delay=True, noisy_delay_threshold=0.2)
    a = pr.run(plans[:, :half], per_episode=True, n_scenarios=half, episode=5, noisy_delay=True,
               noisy_delay_threshold=0.2)
    b = pr.run(plans[:, half:], per_episode=True, n_scenarios=S - half, scenario_offset=half, episode=5,
               noisy_delay=True, noisy_delay_threshold=0.2)
    for k in STATS + ("rewards",):
        np.testing.assert_array_equal(torch.cat([a[k], b[k]], 1).cpu().numpy(), whole[k].cpu().numpy(), err_msg=k)
    pr.close()


def drawn_plan_case(seed, i):
    """One drawn plan-replay case (class i % 4, capacity scale by i): returns (kernel outputs as NumPy,
    oracle outputs, kind). Shared by test_plan_replay_drawn_configs_vs_oracle and
    tools/fuzz_plan_campaign.py."""
    from fuzz_configs import maybe_order_max, rand_config
    rs = np.random.RandomState(seed)
    # the LP scripts replay through raw-state envs (standardise_state False, SHLP_8.py:737-766); a plan
    # rollout sums the raw state, so standardised-state specs (and MAIM_div, whose observations are
    # always scaled) are refused (test_plan_replay_errors)
    kind = ("IM", "IM_div", "MAIM", "IM_div")[i % 4]
    cfg = maybe_order_max(rs, kind, rand_config(rs, kind, (i + i // 4) % 4))   # capacities 5-450
    cfg["standardise_state"] = False
    if kind == "MAIM":
        cfg["independent"] = False           # the rollout needs a scalar reward
    top = float(np.max(cfg["inv_max"]))
    if i % 3 == 2:
        lo = int(rs.randint(0, max(2, int(top // 4))))
        cfg.update(demand_dist="uniform", lower_upper=(lo, lo + 2 + int(rs.randint(0, max(2, int(top // 2))))))
    else:
        cfg.update(demand_dist="poisson", mu=float(np.round(rs.uniform(0.05, 0.5) * top, 1)))
    if kind in ("IM_div", "MAIM_div") and rs.rand() < 0.5:
        cfg.update(noisy_demand=True, noisy_demand_threshold=0.25)
    thr = 0.3 if rs.rand() < 0.5 else 0.0
    N = cfg.get("num_stages", cfg.get("num_nodes"))
    T = cfg["num_periods"]
    P, S, off, ep = 2, 256 + 37, int(rs.randint(0, 1 << 20)), int(rs.randint(0, 50))
    per_episode = bool(i % 2)
    shape = (P, S, T, N) if per_episode else (P, T, N)
    std = cfg.get("standardise_actions", True) or kind == "MAIM_div"
    if std:
        a, b = cfg.get("a", -1.0), cfg.get("b", 1.0)
        plans = rs.uniform(a - 0.3 * (b - a), b + 0.3 * (b - a), size=shape)
    else:
        plans = rs.uniform(-0.2 * top, 1.2 * top, size=shape)
    if rs.rand() < 0.5:
        plans = plans.astype(np.float32)
    pr = _pr(kind, cfg)
    out = pr.run(plans, n_scenarios=S, scenario_offset=off, episode=ep, per_episode=per_episode,
                 noisy_delay=thr > 0, noisy_delay_threshold=thr)
    got = {k: out[k].cpu().numpy() for k in STATS + ("rewards",)}
    pr.close()
    rng = dict(seed=cfg["seed"], episode=ep, env_offset=off, dist=cfg["demand_dist"], mu=cfg.get("mu", 5),
               lower_upper=cfg.get("lower_upper", (1, 5)))
    ref_plans = np.transpose(plans, (2, 0, 1, 3)) if per_episode else plans
    ref = pl.plan_rollout(kind, cfg, ref_plans.astype(np.float64), per_episode=per_episode, n_scenarios=S, rng=rng,
                          noisy_delay=thr > 0, noisy_delay_threshold=thr)
    ref["rewards"] = np.transpose(ref["rewards"], (1, 2, 0))
    return got, ref, kind


@pytest.mark.parametrize("i", range(8))
def test_plan_replay_drawn_configs_vs_oracle(i):
    """Plan replays on drawn configurations of all four classes (tests/fuzz_configs.py: 2-8 stages,
    random trees, capacities 5-450 (uint8 and int16 state), delays 1-5, horizons 10-50, raw or
    standardised actions, shared rewards for the multi-agent classes, explicit order_max), in-kernel
    Poisson / uniform demand, noisy demand on trees, noisy delay; float32 or float64 plans drawn around
    the action range (standardised: beyond [a, b]; raw: beyond [0, order_max], fractional). Every
    per-episode value and per-step reward equals the oracle."""
    got, ref, _ = drawn_plan_case(9090 + i, i)
    for k in STATS + ("rewards",):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)

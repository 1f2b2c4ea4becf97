"""Handles past every 32-bit offset boundary, exact against the oracle on slices that straddle them.

imenv_create accepts up to 2^31 envs per handle (include/imenv.h). These runs use handles large
enough that the step kernel's element offsets pass 2^31 and its byte offsets pass 2^32. That holds for
observations, actions and (C2) rewards. A 32-bit index anywhere on those paths would put the envs
past the boundary on the wrong rows. C2 runs 2^29 + 4,096 envs (about 47 GB in all) and 2^31 (the
ABI's maximum, about 210 GB). C4 (the tree, with history observations) runs 2^28 + 4,096 (about 45
GB). For each boundary, a 256-env slice that straddles it is checked over a whole episode against the
oracle under the same Philox keys. In-kernel demand, float32 actions; the JIT and the ahead-of-time
kernels both run.
"""
import numpy as np
import pytest
import torch

from oracle.im_oracle import OracleEnv

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

C2 = dict(num_stages=4, num_periods=30, init_inv=np.ones(4) * 10, inv_target=np.zeros(4),
          inv_max=np.ones(4) * 30, price=np.array([5, 4, 3, 2, 1]),
          stock_cost=np.array([0.35, 0.3, 0.4, 0.2]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.9]),
          delay=np.array([1, 2, 3, 1]), demand_dist="poisson", mu=5, seed=52, independent=False)
C4 = dict(num_nodes=4, connections={0: [1], 1: [2, 3], 2: [], 3: []}, num_periods=30,
          init_inv=np.ones(4) * 10, inv_target=np.zeros(4), inv_max=np.ones(4) * 30,
          stock_cost=np.array([0.35, 0.3, 0.4, 0.4]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.6]),
          delay=np.array([1, 2, 1, 1]), demand_dist="poisson", mu=5, seed=52, time_dependency=True,
          prev_demand=True, independent=False)


def boundary_slices(n, row_bytes, act_bytes=16, rew_bytes=8, width=256):
    """Slices of `width` envs around every env whose observation / action / reward element or byte
    offset first reaches 2^31 or 2^32, plus both ends of the batch."""
    starts = {0, n - width}
    for per_env in (row_bytes, act_bytes, rew_bytes):
        for elem in (4, 8):
            if per_env % elem:
                continue
            for lim in (1 << 31, 1 << 32):
                for unit in (elem, 1):          # element index, byte offset
                    e = -(-lim * unit // per_env)  # first env at or past the boundary
                    if 0 < e < n:
                        starts.add(min(max(e - width // 2, 0), n - width))
    return sorted(starts)


@pytest.mark.parametrize("kind,cfg,n,mode", [
    ("MAIM", C2, (1 << 29) + 4096, "jit"), ("MAIM", C2, (1 << 29) + 4096, "aot"),
    ("MAIM_div", C4, (1 << 28) + 4096, "jit"), ("MAIM_div", C4, (1 << 28) + 4096, "aot"),
    ("MAIM", C2, 1 << 31, "jit")])         # the largest handle imenv_create accepts (about 210 GB here)
def test_offsets_past_32_bits_match_oracle(kind, cfg, n, mode):
    from imenv import VectorInvEnv
    free = _free_bytes()
    env = VectorInvEnv(kind, cfg, n_envs=n, device=DEV)
    env.set_jit(1 if mode == "jit" else 0)
    N, F = env.N, env.F
    need = n * (N * 4 + N * F * 4 + 8 + 32)      # actions, observations, rewards, state + error flags
    if free < 1.1 * need:
        env.close()
        pytest.skip("needs %.0f GB of free device memory, %.0f GB free" % (need / 2**30, free / 2**30))
    obs = torch.empty((n, N, F), dtype=torch.float32, device=DEV)
    rew = torch.empty(env.reward_shape(), dtype=torch.float64, device=DEV)
    act = torch.empty((n, N), dtype=torch.float32, device=DEV)
    starts = boundary_slices(n, N * F * 4, act_bytes=N * 4, rew_bytes=rew[0].numel() * 8)
    assert len(starts) >= 4
    k = 256
    oras = [OracleEnv(kind, cfg, n_envs=k) for _ in starts]
    env.reset(obs_out=obs)
    for s, ora in zip(starts, oras):
        r0 = ora.reset(rng=dict(seed=52, episode=0, env_offset=s, dist="poisson", mu=5))
        np.testing.assert_array_equal(obs[s:s + k].cpu().numpy(), r0.astype(np.float32), err_msg="reset @%d" % s)
    g = torch.Generator(device=DEV)
    g.manual_seed(11)
    for t in range(30):
        torch.rand((n, N), generator=g, device=DEV, out=act)
        act.mul_(2.2).sub_(1.1)
        env.step(act, obs_out=obs, reward_out=rew)
        for s, ora in zip(starts, oras):
            o_c, r_c, _, _ = ora.step(act[s:s + k].double().cpu().numpy())
            np.testing.assert_array_equal(obs[s:s + k].cpu().numpy(), o_c.astype(np.float32),
                                          err_msg="%s obs t=%d @%d" % (kind, t, s))
            np.testing.assert_array_equal(rew[s:s + k].cpu().numpy(), r_c, err_msg="%s reward t=%d @%d" % (kind, t, s))
    flags, anyv = env.errors()
    assert anyv == 0
    env.close()
    del obs, rew, act
    torch.cuda.empty_cache()


def _free_bytes():
    torch.cuda.empty_cache()
    return torch.cuda.mem_get_info(DEV)[0]


@pytest.mark.parametrize("kind,base", [("IM", "serial4"), ("IM_div", "div1")])
def test_plan_replay_offsets_past_32_bits(kind, base):
    """Plan replay with one float64 plan per scenario over 2^25 + 256 scenarios. The plans' element
    offsets pass 2^31 and their byte offsets 2^32 from period 4 on; the per-step reward rows pass 2^32
    bytes too. Scenario slices across the batch are checked against the oracle's replay under the
    same keys. The plans are made on the device, already in the kernel's [T][P][S][N] layout, and
    handed over as a [P][S][T][N] view, so no transposed copy is made."""
    import gen_cfg
    from oracle import plan as pl
    from imenv.plan import PlanRollout
    cfg = gen_cfg.__dict__[base](standardise_state=False, standardise_actions=False)
    N, T, S = cfg.get("num_stages", cfg.get("num_nodes")), cfg.get("num_periods", 30), (1 << 25) + 256
    need = S * (T * N * 8 + T * 8 + 5 * 8) + (1 << 30)
    if _free_bytes() < 1.1 * need:
        pytest.skip("needs %.0f GB of free device memory" % (need / 2**30))
    g = torch.Generator(device=DEV)
    g.manual_seed(4)
    x = torch.randint(0, 25, (T, 1, S, N), generator=g, device=DEV).to(torch.float64)
    x += 0.5 * torch.randint(0, 2, (T, 1, S, N), generator=g, device=DEV)
    pr = PlanRollout(kind, cfg, device=DEV)
    out = pr.run(x.permute(1, 2, 0, 3), per_episode=True, n_scenarios=S, episode=1)
    for s in (0, S // 3, S // 2 + 77, S - 256):
        k = 256
        rng = dict(seed=cfg["seed"], episode=1, env_offset=s, dist="poisson", mu=cfg.get("mu", 5))
        ref = pl.plan_rollout(kind, cfg, x[:, :, s:s + k].cpu().numpy(), per_episode=True, n_scenarios=k, rng=rng)
        for name in ("return", "inventory", "backlog", "customer_backlog"):
            np.testing.assert_array_equal(out[name][:, s:s + k].cpu().numpy(), ref[name], err_msg="%s @%d" % (name, s))
        np.testing.assert_array_equal(out["rewards"][:, s:s + k].cpu().numpy(), np.transpose(ref["rewards"], (1, 2, 0)),
                                      err_msg="rewards @%d" % s)
    pr.close()
    del x, out
    torch.cuda.empty_cache()


def test_base_stock_rollout_offsets_past_32_bits():
    """128 base-stock policies x (2^22 + 64) drawn scenarios in one launch (1.6e10 env-steps): the
    per-episode output rows ([stat][P][S] float64) pass 2^31 elements and 2^32 bytes. (policy,
    scenario) slices across the batch equal the oracle's rollout under the same keys."""
    import gen_cfg
    from scipy.stats import poisson
    from oracle import base_stock as bs
    from imenv.policy import BaseStockRollout
    cfg = gen_cfg.serial4(standardise_state=False, standardise_actions=False)
    P, S = 128, (1 << 22) + 64
    need = 5 * P * S * 8 + (1 << 30)
    if _free_bytes() < 1.1 * need:
        pytest.skip("needs %.0f GB of free device memory" % (need / 2**30))
    pol = np.random.RandomState(9).uniform(0, 50, size=(P, 4))
    ro = BaseStockRollout("IM", cfg, device=DEV)
    out = ro.run(pol, n_scenarios=S, episode=6)
    for p, s in ((0, 0), (127, S - 200), (64, S // 2), (100, 12345), (31, S - 4000)):
        k = 200
        rng = dict(seed=cfg["seed"], episode=6, env_offset=s, dist="poisson", mu=5)
        ref = bs.rollout("IM", cfg, pol[p:p + 1], n_scenarios=k, rng=rng, pmf=lambda v: poisson.pmf(v, mu=5))
        for name in ("return", "objective", "inventory", "backlog", "customer_backlog"):
            np.testing.assert_array_equal(out[name][p, s:s + k].cpu().numpy(), ref[name][0],
                                          err_msg="%s (%d, %d)" % (name, p, s))
    ro.close()
    del out
    torch.cuda.empty_cache()


def test_gae_and_cc_observation_offsets_past_32_bits():
    """GAE over a [30, 2^27 + 64] buffer (4.0e9 elements per row array) and centralised-critic rows
    for [2^26 + 64] envs x 4 agents (4.0e9 output elements): sampled envs at the start, across the
    2^31-element boundaries and at the end equal the oracle restatements."""
    from oracle.gae import gae_batch
    from oracle.cc_obs import cc_observation as cc_ref
    from imenv.rollout import gae
    from imenv.critic import cc_observation
    T, n = 30, (1 << 27) + 64
    need = T * n * (8 + 4 + 4 + 4) + (1 << 30)
    if _free_bytes() < 1.1 * need:
        pytest.skip("needs %.0f GB of free device memory" % (need / 2**30))
    g = torch.Generator(device=DEV)
    g.manual_seed(12)
    r = torch.randn((T, n), generator=g, device=DEV, dtype=torch.float64) * 30
    v = torch.randn((T, n), generator=g, device=DEV) * 100
    adv, vt = gae(r, v)
    cols = np.unique(np.concatenate([np.arange(0, 64), np.arange(n - 64, n),
                                     np.arange(-64, 64) + (1 << 31) // T, np.arange(-64, 64) + (1 << 32) // (4 * T),
                                     np.random.RandomState(1).randint(0, n, 256)]))
    idx = torch.as_tensor(cols, device=DEV)
    ea, ev = gae_batch(r[:, idx].cpu().numpy(), v[:, idx].cpu().numpy())
    np.testing.assert_array_equal(adv[:, idx].cpu().numpy(), ea)
    np.testing.assert_array_equal(vt[:, idx].cpu().numpy(), ev)
    del r, v, adv, vt
    torch.cuda.empty_cache()

    m = (1 << 26) + 64                    # CC rows: [m, 4, 15] float32 = 4.0e9 elements
    obs = torch.rand((m, 4, 3), generator=g, device=DEV) * 2 - 1
    act = torch.rand((m, 4), generator=g, device=DEV) * 3 - 1.5
    got = cc_observation(obs, act)
    assert got.shape == (m, 4, 15)
    rows = np.unique(np.concatenate([np.arange(0, 64), np.arange(m - 64, m),
                                     np.arange(-64, 64) + (1 << 31) // 60, np.arange(-64, 64) + (1 << 32) // 240,
                                     np.random.RandomState(2).randint(0, m, 256)]))
    ri = torch.as_tensor(rows, device=DEV)
    exp = cc_ref(obs[ri].cpu().numpy(), act[ri].cpu().numpy())
    np.testing.assert_array_equal(got[ri].cpu().numpy(), exp)
    del obs, act, got
    torch.cuda.empty_cache()


def test_column_stats_offsets_past_32_bits():
    """The evaluation harness's column statistics (imenv_column_stats) over a (2^28 + 12,345) x 8
    float64 matrix (2^31 + 98,760 elements, 17 GB): every column's mean and std equal a float64
    torch reduction of the same matrix within 1e-10 relative (means also 1e-9 absolute)."""
    from imenv import _native as nat
    rows, cols = (1 << 28) + 12345, 8
    if _free_bytes() < 1.2 * rows * cols * 8 + (1 << 30):
        pytest.skip("needs %.0f GB of free device memory" % (rows * cols * 8 / 2**30))
    g = torch.Generator(device=DEV)
    g.manual_seed(13)
    x = torch.randn((rows, cols), generator=g, dtype=torch.float64, device=DEV)
    x.mul_(torch.arange(1, cols + 1, device=DEV, dtype=torch.float64) * 7).add_(torch.arange(cols, device=DEV) * 3.0)
    x[-1] = 1e6                          # the last row (past the 2^31-element mark) must be counted
    out = torch.empty((cols, 2), dtype=torch.float64, device=DEV)
    nat.check(nat.load().imenv_column_stats(x.data_ptr(), rows, cols, out.data_ptr(), None), "column_stats")
    torch.cuda.synchronize()
    mean = x.mean(dim=0)
    std = x.std(dim=0, correction=0)
    np.testing.assert_allclose(out[:, 0].cpu().numpy(), mean.cpu().numpy(), rtol=1e-10, atol=1e-9)
    np.testing.assert_allclose(out[:, 1].cpu().numpy(), std.cpu().numpy(), rtol=1e-10)
    del x
    torch.cuda.empty_cache()

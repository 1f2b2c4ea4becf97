"""BASELINE.json's GPU configs at their full sizes, exact against the oracle over a whole episode.

C2: MultiAgentInvManagement 4-stage, 65,536 envs. C3: 8-stage serial chain (SHLP_8 constants),
262,144 envs. C4: divergent div1 network with MA_6 flags, 131,072 envs. Demand is drawn in-kernel
(Philox, keyed by global env id; the oracle's twin draws the same values), actions are float32.
Every period compares inventory / backlog / unfulfilled orders bit-exactly, observations as float32
and rewards as float64 bit-exactly, for every env.
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
C3 = dict(num_stages=8, num_periods=30, init_inv=np.ones(8) * 10, inv_target=np.zeros(8),
          inv_max=np.ones(8) * 30, price=np.array([9, 8, 7, 6, 5, 4, 3, 2, 1]),
          stock_cost=np.array([0.35, 0.3, 0.4, 0.2, 0.35, 0.3, 0.4, 0.2]),
          backlog_cost=np.array([0.5, 0.7, 0.6, 0.9, 0.5, 0.7, 0.6, 0.9]),
          delay=np.array([1, 2, 3, 1, 4, 2, 3, 1]), demand_dist="poisson", mu=5, seed=52)
C4 = dict(num_nodes=4, connections={0: [1], 1: [2, 3], 2: [], 3: []}, num_periods=30,
          init_inv=np.ones(4) * 10, inv_target=np.zeros(4), inv_max=np.ones(4) * 30,
          stock_cost=np.array([0.35, 0.3, 0.4, 0.4]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.6]),
          delay=np.array([1, 2, 1, 1]), demand_dist="poisson", mu=5, seed=52, time_dependency=True,
          prev_demand=True, independent=False)


@pytest.mark.parametrize("name,kind,cfg,n", [("C2", "MAIM", C2, 65536), ("C3", "IM", C3, 262144),
                                             ("C4", "MAIM_div", C4, 131072)])
def test_full_size_episode_matches_oracle(name, kind, cfg, n):
    from imenv import VectorInvEnv
    env = VectorInvEnv(kind, cfg, n_envs=n, device=DEV)
    ora = OracleEnv(kind, cfg, n_envs=n)
    o_g = env.reset()
    o_c = ora.reset(rng=dict(seed=52, episode=0, env_offset=0, dist="poisson", mu=5))
    np.testing.assert_array_equal(o_g.cpu().numpy(), o_c.astype(np.float32))
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    for t in range(30):
        a = torch.rand((n, env.N), generator=g, device=DEV, dtype=torch.float32) * 2.2 - 1.1
        o_g, r_g, d_g, _ = env.step(a)
        o_c, r_c, d_c, _ = ora.step(a.cpu().numpy().astype(np.float64))
        st = env.state()
        ref = ora.state_arrays()
        for k in ("inv", "backlog", "order_u"):
            np.testing.assert_array_equal(st[k].cpu().numpy(), ref[k], err_msg="%s %s t=%d" % (name, k, t))
        np.testing.assert_array_equal(o_g.cpu().numpy(), o_c.astype(np.float32), err_msg="%s obs t=%d" % (name, t))
        np.testing.assert_array_equal(r_g.cpu().numpy(), r_c, err_msg="%s reward t=%d" % (name, t))
        assert d_g == d_c
    flags, anyv = env.errors()
    assert anyv == 0
    assert "jit:" in env.kernel_info()
    env.close()

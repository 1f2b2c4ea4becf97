"""Drawn demand (IMENV_LAYOUT_DRAW: in-kernel Philox, Poisson or uniform, noisy demand on trees) on drawn
specifications: the GPU step kernel against the oracle's Philox twin over two episodes, with the
drawn-demand hand-over table forced on (every retailer count: the step at t % 4 == 0 parks periods
t+1..t+3, imenv_draw_layout) with the hipRTC kernel, and at the default (on for single-retailer handles
of <= 131,072 envs) with the ahead-of-time kernel (no compile per case).
Episode lengths 10 / 30 / 50 end inside a Philox block (T % 4 == 2), ragged env counts leave tail lanes.
Parity is bit-exact (state, float32 observations, float64 rewards); the oracle's Philox twin is pinned
by Random123's known-answer vectors (tests/test_philox.py)."""
import numpy as np
import pytest
import torch

import test_gpu_parity as tp
from fuzz_configs import rand_config

pytestmark = pytest.mark.gpu

KINDS = ["IM", "MAIM", "IM_div", "MAIM_div"]


def make_drawn_case(i):
    rs = np.random.RandomState(700000 + i)
    kind = KINDS[i % 4]
    cfg = rand_config(rs, kind, i)
    if rs.rand() < 0.6:
        cfg.update(demand_dist="poisson", mu=float(np.round(rs.uniform(1.0, 40.0), 1)))
    else:
        lo = int(rs.randint(0, 50))
        cfg.update(demand_dist="uniform", lower_upper=(lo, lo + int(rs.choice([3, 40, 600]))))
    if kind.endswith("_div") and rs.rand() < 0.5:
        cfg.update(noisy_demand=True, noisy_demand_threshold=float(rs.choice([0.1, 0.3, 0.6])))
    n = int(rs.choice([64, 200, 256, 1000]))
    return kind, cfg, n


def rng_of(cfg, ep, off):
    return dict(seed=cfg["seed"], episode=ep, env_offset=off, dist=cfg["demand_dist"], mu=cfg.get("mu", 5),
                lower_upper=cfg.get("lower_upper", (1, 5)))


@pytest.mark.parametrize("dtab,kernel", [("1", "jit"), ("default", "aot")])
@pytest.mark.parametrize("i", range(16))
def test_gpu_drawn_demand_random_spec_matches_oracle(i, dtab, kernel, monkeypatch):
    from oracle.im_oracle import OracleEnv
    if dtab == "1":
        monkeypatch.setenv("IMENV_DTAB", "1")
    else:
        monkeypatch.delenv("IMENV_DTAB", raising=False)
    kind, cfg, n = make_drawn_case(i)
    off = 37 * i
    env = tp._env(kind, cfg, n, env_offset=off)
    env.set_jit(1 if kernel == "jit" else 0)
    # the split's round-robin a phase at a time (pinned equal to the literal loops by
    # tests/test_split_closed_form.py): capacities of ~40,000 take minutes per episode in the literal loops
    ora = OracleEnv(kind, cfg, n_envs=n, split="closed")
    if dtab == "1":
        assert env.draw_layout() > 0
    else:
        assert (env.draw_layout() > 0) == (env.spec.num_retailers == 1)
    T = env.T
    rs = np.random.RandomState(i)
    for ep in range(2):
        env.reset()
        ora.reset(rng=rng_of(cfg, ep, off))
        for t in range(T):
            a = rs.uniform(-1.2, 1.2, size=(n, env.N))
            o_g, r_g, _, _ = env.step(torch.as_tensor(a, device=tp.DEV))
            o_c, r_c, _, _ = ora.step(a)
            msg = "case %d %s ep %d t %d" % (i, kind, ep, t)
            np.testing.assert_array_equal(o_g.cpu().numpy(), o_c.astype(np.float32), err_msg=msg)
            np.testing.assert_array_equal(r_g.cpu().numpy(), r_c, err_msg=msg)
        st = env.state()
        for k in ("inv", "backlog", "order_u"):
            np.testing.assert_array_equal(st[k].cpu().numpy(), ora.state_arrays()[k], err_msg="%s %s" % (k, msg))
    assert ("jit:" in env.kernel_info()) == (kernel == "jit")
    env.close()

"""VectorInvEnv's API surface on drawn configurations, against the oracle.

Each case draws a configuration (tests/fuzz_configs.py) and a way of driving it: batch size
(1 to 300 envs, ragged), env_offset, demand mode (per-env host table, one broadcast table, or
in-kernel Philox draws of Poisson / uniform demand, with noisy demand on trees), noisy delay (host
uniforms or in-kernel draws), float32 or float64 actions and observations, info=True, info_out=
buffers and state() read-backs at random periods, two episodes on one handle. Everything the
calls return is compared with the oracle bit for bit (float32 observations with the oracle's
float64 value rounded to float32). A configuration the hand-written tests never formed is how the
custom-demand default bug (a [1, T] table taken for per-env demand) was found.
"""
import numpy as np
import pytest
import torch

from fuzz_configs import rand_config
from oracle.im_oracle import OracleEnv

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
KINDS = ["IM", "MAIM", "IM_div", "MAIM_div"]
INFO_KEYS = ("order", "demand", "acquisition", "ship", "profit", "ship_to", "backlog_to")


def _case(i):
    rs = np.random.RandomState(777 + i)
    kind = KINDS[i % 4]
    cfg = rand_config(rs, kind, (i // 4) % 4)
    tree = kind.endswith("div")
    mode = ["per_env", "broadcast", "drawn"][i % 3]
    if mode == "drawn":
        top = float(np.max(cfg["inv_max"]))
        if rs.rand() < 0.5:
            cfg.update(demand_dist="poisson", mu=float(np.round(rs.uniform(0.05, 0.6) * top, 1)))
        else:
            lo = int(rs.randint(0, max(2, int(top // 4))))
            cfg.update(demand_dist="uniform", lower_upper=(lo, lo + 2 + int(rs.randint(0, max(2, int(top // 2))))))
        if tree and rs.rand() < 0.5:
            cfg.update(noisy_demand=True, noisy_demand_threshold=float(np.round(rs.uniform(0.05, 0.4), 2)))
    n = int(rs.choice([1, 7, 64, 300]))
    noisy = float(np.round(rs.uniform(0.1, 0.5), 2)) if rs.rand() < 0.4 else 0.0
    host_u = bool(rs.rand() < 0.5) or mode != "drawn"        # in-kernel noisy delay needs drawn keys
    return rs, kind, cfg, mode, n, noisy, host_u


@pytest.mark.parametrize("i", range(24))
def test_gpu_api_on_drawn_configs(i):
    from imenv import VectorInvEnv
    rs, kind, cfg, mode, n, noisy, host_u = _case(i)
    serial = kind in ("IM", "MAIM")
    odt = torch.float64 if rs.rand() < 0.5 else torch.float32
    adt = torch.float64 if rs.rand() < 0.5 else torch.float32
    off = int(rs.randint(0, 1 << 20))
    env = VectorInvEnv(kind, cfg, n_envs=n, device=DEV, obs_dtype=odt, env_offset=off)
    ora = OracleEnv(kind, cfg, n_envs=n)
    N, T, R = env.N, env.T, env.R
    top = int(np.max(cfg["inv_max"]))
    for ep in range(2):
        kw, okw = {}, {}
        if mode == "per_env":
            dem = rs.randint(0, top + 1, size=(n, T) if serial else (n, R, T))
            kw["customer_demand"] = okw["customer_demand"] = dem
        elif mode == "broadcast":
            dem = rs.randint(0, top + 1, size=(T,) if serial else (R, T))
            kw["customer_demand"] = okw["customer_demand"] = dem
        else:
            okw["rng"] = dict(seed=cfg["seed"], episode=ep, env_offset=off, dist=cfg["demand_dist"],
                              mu=cfg.get("mu", 5), lower_upper=cfg.get("lower_upper", (1, 5)))
        if noisy:
            kw.update(noisy_delay=True, noisy_delay_threshold=noisy)
            okw.update(noisy_delay=True, noisy_delay_threshold=noisy)
            if host_u:
                u = rs.uniform(0, 1, size=(n, T, N))
                kw["delay_uniforms"] = okw["delay_uniforms"] = u
        o_g = env.reset(**kw)
        o_c = ora.reset(**okw)
        np.testing.assert_array_equal(o_g.cpu().numpy(), o_c.astype(o_g.cpu().numpy().dtype))
        for t in range(T):
            a = rs.uniform(env.spec.a - 0.3, env.spec.b + 0.3, size=(n, N)) if env.spec.standardise_actions \
                else rs.uniform(-2, 1.2 * top, size=(n, N))
            at = torch.as_tensor(a, device=DEV, dtype=adt)
            a_ref = at.double().cpu().numpy()
            how = rs.randint(3)
            if how == 0:
                o_g, r_g, d_g, inf = env.step(at, info=True)
            elif how == 1:
                inf = {k: torch.empty((n, N), dtype=torch.float64 if k == "profit" else torch.int32, device=DEV)
                       for k in INFO_KEYS}
                o_g, r_g, d_g, _ = env.step(at, info_out=inf)
            else:
                o_g, r_g, d_g, inf = env.step(at)
            o_c, r_c, d_c, inf_c = ora.step(a_ref)
            msg = "case %d ep %d t %d" % (i, ep, t)
            np.testing.assert_array_equal(o_g.cpu().numpy(), o_c.astype(o_g.cpu().numpy().dtype), err_msg=msg)
            np.testing.assert_array_equal(r_g.cpu().numpy(), r_c, err_msg=msg)
            assert d_g == d_c
            if inf is not None:
                for k in ("order", "demand", "acquisition", "ship", "profit"):
                    np.testing.assert_array_equal(inf[k].cpu().numpy().astype(np.float64), inf_c[k],
                                                  err_msg=msg + " " + k)
            if rs.rand() < 0.3:
                st = env.state()
                for k in ("inv", "backlog", "order_u"):
                    np.testing.assert_array_equal(st[k].cpu().numpy(), ora.state_arrays()[k], err_msg=msg + " " + k)
    flags, anyv = env.errors()
    assert anyv == 0 and not ora.err.any()
    env.close()

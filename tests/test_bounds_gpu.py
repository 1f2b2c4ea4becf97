"""State values driven to their proven bounds (the range the JIT observation closed forms are verified
over: imenv_jit.hip emit_obs_hooks, vbound = state_bound) stay bit-exact against the oracle.

Demand is set at every retailer's capacity and the actions order nothing (or everything), so
backlogs climb to their caps (IM_div_env.py / MAIM_div_env.py: demand_max; serial: inv_max when
standardised), order_u and in-transit slots reach their maxima, and noisy delay piles deferred
arrivals into the carry. Every observation value (float32 and float64), reward and state row is
compared for every env and period, and the test checks that the bounds were actually reached."""
import numpy as np
import pytest
import torch

from golden_io import load_case
from oracle.im_oracle import OracleEnv

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("name", ["C2_MAIM4", "C4_MAIM_div1", "IM_div1_td_pd_pa", "MAIM4_all_L2", "MAIM_div2_share"])
@pytest.mark.parametrize("odt", [torch.float32, torch.float64])
@pytest.mark.parametrize("noisy", [0.0, 0.5])
def test_saturated_backlogs_and_pipelines(name, odt, noisy):
    from imenv import VectorInvEnv
    meta, _ = load_case(name)
    kind, cfg = meta["kind"], meta["config"]
    E = 256
    env = VectorInvEnv(kind, cfg, n_envs=E, device=DEV, obs_dtype=odt)
    ora = OracleEnv(kind, cfg, n_envs=E)
    N, T, R = env.N, env.T, env.R
    serial = kind in ("IM", "MAIM")
    cap = np.asarray(env.spec.inv_max)
    rs = np.random.RandomState(3)
    # retailer demand at (and a little over) its capacity every period
    dem = np.full((E, T) if serial else (E, R, T), int(cap.max()) + 3)
    u = rs.uniform(0, 1, (E, T, N)) if noisy else None
    kw = dict(customer_demand=dem, noisy_delay=bool(noisy), noisy_delay_threshold=noisy)
    o_g = env.reset(delay_uniforms=u, **kw)
    o_c = ora.reset(delay_uniforms=u, **kw)
    np.testing.assert_array_equal(o_g.cpu().numpy(), o_c.astype(o_g.cpu().numpy().dtype))
    a_lo, a_hi = env.spec.a, env.spec.b
    max_bl = np.zeros(N)
    for t in range(T):
        # first half: order nothing (backlogs climb to their caps); then order everything
        a = np.full((E, N), a_lo if t < T // 2 else a_hi, dtype=np.float64)
        a[::7] = rs.uniform(a_lo, a_hi, (len(a[::7]), N))
        o_g, r_g, _, _ = env.step(torch.as_tensor(a, device=DEV))
        o_c, r_c, _, _ = ora.step(a)
        st, ref = env.state(), ora.state_arrays()
        for k in ("inv", "backlog", "order_u"):
            np.testing.assert_array_equal(st[k].cpu().numpy(), ref[k], err_msg="%s t=%d" % (k, t))
        np.testing.assert_array_equal(o_g.cpu().numpy(), o_c.astype(o_g.cpu().numpy().dtype), err_msg="obs t=%d" % t)
        np.testing.assert_array_equal(r_g.cpu().numpy(), r_c, err_msg="reward t=%d" % t)
        max_bl = np.maximum(max_bl, ref["backlog"].max(axis=0))
    # the retailers' backlogs did reach their caps (the top of the verified observation range)
    bcap = np.asarray(env.spec.backlog_cap)
    ret = [r for r in env.spec.retailers if bcap[r] >= 0]
    assert ret and all(max_bl[r] == bcap[r] for r in ret), (max_bl, bcap, env.spec.retailers)
    assert env.kernel_info().startswith("jit:")
    env.close()

"""GPU step kernels vs the oracle on randomly drawn specifications.

The oracle is pinned to the reference on the committed fixtures, which include 26 drawn
configurations (tests/golden/fuzz), and tools/fuzz_explore.py ran it against the reference on 1,400
more drawn configurations without a mismatch. This test carries that coverage to the kernels:
32 further drawn configurations (tests/fuzz_configs.py: all four classes, 2-8 stages or random
trees, capacities 5-450, explicit order_max, delays 1-5, horizons 10-50, every observation flag,
standardised or raw, shared or independent rewards, noisy delay with host uniforms) x 64 envs, on
the hipRTC-specialised and the ahead-of-time kernels. Integer state and every info field, float64
observations and rewards: bit-exact.
"""
import numpy as np
import pytest

import test_gpu_parity as tp
from fuzz_configs import fuzz_inputs, maybe_order_max, rand_config
from test_oracle_golden import run_oracle

pytestmark = pytest.mark.gpu
KINDS = ["IM", "MAIM", "IM_div", "MAIM_div"]
NUM = 32
E = 64


def make_case(i):
    rs = np.random.RandomState(90000 + i)
    kind = KINDS[i % 4]
    cfg = rand_config(rs, kind, (i // 4) % 4)      # capacity scales 30, 120, 5, 300
    cfg = maybe_order_max(rs, kind, cfg)
    noisy = 0.3 if rs.rand() < 0.3 else 0.0
    dem, act, unif = fuzz_inputs(kind, cfg, {}, 90000 + i, E)
    meta = dict(kind=kind, config=cfg, noisy=noisy, E=E, T=cfg["num_periods"])
    d = dict(customer_demand=dem, actions=act, delay_uniforms=unif if noisy else np.zeros((0,)))
    return meta, d


@pytest.mark.parametrize("mode", ["jit", "aot"])
@pytest.mark.parametrize("i", range(NUM))
def test_gpu_random_spec_matches_oracle(i, mode):
    meta, d = make_case(i)
    obs0_o, out_o, env_o = run_oracle(meta, d)
    tp.MODE["kernel"] = mode
    obs0_g, out_g, anyerr = tp.run_gpu_case(meta, d)
    assert anyerr == 0 and not env_o.err.any()
    np.testing.assert_array_equal(obs0_g, obs0_o)
    keys = ["order", "demand", "acquisition", "ship", "inv", "backlog", "order_u", "profit", "obs"]
    if meta["kind"] in ("IM_div", "MAIM_div"):
        keys += ["ship_to", "backlog_to"]
    for k in keys:
        np.testing.assert_array_equal(out_g[k].astype(np.float64), out_o[k], err_msg="%d/%s" % (i, k))
    np.testing.assert_array_equal(out_g["reward"], out_o["reward"])

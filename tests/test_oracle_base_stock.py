"""Pin the base-stock restatement (oracle/base_stock.py) against the reference's own outputs.

tests/golden/base_stock.npz was produced by running base_restock_policy.py's dfo_func /
base_stock_policy / optimize_inventory_policy on the reference env classes
(tools/gen_base_stock_fixtures.py). Every comparison is exact: the objective, per-step rewards and
episode returns are float64-bit-equal, the state sums integer-equal.
"""
import numpy as np
import pytest
from scipy.optimize import minimize
from scipy.stats import poisson, randint

from golden_io import load_base_stock
from oracle import base_stock as bs
from oracle.im_oracle import OracleEnv

META, CASES = load_base_stock()
ROLL = [c for c in CASES if c != "powell"]


def pmf_of(cfg):
    if cfg.get("demand_dist") == "uniform":
        lo, hi = cfg["lower_upper"]
        return lambda k: randint.pmf(k, low=lo, high=hi)
    return lambda k: poisson.pmf(k, mu=cfg.get("mu", 5))


@pytest.mark.parametrize("name", ROLL)
def test_oracle_rollout_matches_reference(name):
    m, d = META[name], CASES[name]
    out = bs.rollout(m["kind"], m["config"], d["policies"], demand=d["demand"], pmf=pmf_of(m["config"]))
    np.testing.assert_array_equal(out["rewards"], d["rewards"])
    np.testing.assert_array_equal(out["return"], d["return"])
    np.testing.assert_array_equal(out["objective"], d["objective"])
    for k in ("inventory", "backlog", "customer_backlog"):
        np.testing.assert_array_equal(out[k], d[k])


def test_oracle_powell_matches_reference():
    """Powell over the restated objective retraces the reference's search exactly."""
    m, d = META["powell"], CASES["powell"]
    cfg = m["config"]
    pmf = pmf_of(cfg)

    def fun(policy):
        return bs.rollout(m["kind"], cfg, policy[None, :], demand=d["demand"][None, :], pmf=pmf)["objective"][0, 0]

    res = minimize(fun=fun, x0=np.array(m["init_policy"]), method="Powell")
    assert res.nfev == int(d["nfev"])
    np.testing.assert_array_equal(res.x, d["x"])
    assert res.fun == float(d["fun"])
    np.testing.assert_array_equal(np.round(np.maximum(res.x, 0), 0).astype(int), d["policy"])


def test_base_stock_policy_formula():
    """base_restock_policy.py:12-20 on hand-made state: echelon position, clamp to [0, order_max]."""
    inv = np.array([[10.0, 0, 5, 30]])
    ou = np.array([[3.0, 7, 0, 0]])
    bl = np.array([[0.0, 4, 0, 0]])
    act = bs.base_stock_policy(np.array([20.0, 2.5, 100.0, 10.0]), inv, ou, bl, np.array([30.0, 30, 30, 30]))
    np.testing.assert_array_equal(act, [[7.0, 0.0, 30.0, 0.0]])


def test_policy_stats_are_numpy_mean_std():
    rs = np.random.RandomState(0)
    per = {k: rs.standard_normal((3, 17)) for k in bs.STAT_NAMES}
    st = bs.policy_stats(per)
    assert st.shape == (3, 5, 2)
    np.testing.assert_array_equal(st[:, 0, 0], per["return"].mean(axis=1))
    np.testing.assert_array_equal(st[:, 4, 1], per["customer_backlog"].std(axis=1))

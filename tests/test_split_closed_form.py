"""Closed forms of the step kernel checked against the reference's own expressions on CPU: the two-child
round robin of the divergent split (csrc/imenv_device.h rr_closed<2>, restated in tools/check_rr_closed.py)
against the literal loop (IM_div_env.py:413-498), guard trips included. The kernels themselves are
pinned against the reference by tests/test_gpu_parity.py and tests/test_fuzz_gpu.py."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

from check_rr_closed import check  # noqa: E402


def test_two_child_round_robin_closed_form_equals_literal_loop():
    n, bad = check(xr=range(-3, 11), ar=range(-2, 25), lims=(0, 1, 2, 4, 7, 60))
    assert n > 50000
    assert not bad, bad[:5]



def test_closed_form_at_the_largest_accepted_guard_limit():
    """imenv_create accepts split guard limits up to 2^30 (tools/asan_host_check.py: 2^30 + 1 and
    INT32_MAX are refused): at 2^30 the int32 closed form still equals the literal loop, while at
    INT32_MAX its `lim + 1` would wrap (the reason for the bound)."""
    n, bad = check(xr=range(-2, 9), ar=range(-2, 20), lims=(1 << 30,))
    assert n > 4000 and not bad, bad[:5]
    _, bad = check(xr=range(1, 4), ar=range(1, 6), lims=(2 ** 31 - 1,))
    assert bad      # documents the overflow that validation prevents


def _oracle_pair(m):
    """Two OracleEnv instances of a tree whose factory has m children (literal / closed split)."""
    import numpy as np
    from oracle.im_oracle import OracleEnv
    conn = {0: list(range(1, m + 1))}
    conn.update({k: [] for k in range(1, m + 1)})
    N = m + 1
    cfg = dict(num_nodes=N, connections=conn, num_periods=10, init_inv=np.ones(N) * 10, inv_target=np.zeros(N),
               inv_max=np.ones(N) * 30, stock_cost=np.ones(N) * 0.1, backlog_cost=np.ones(N) * 0.2,
               delay=np.ones(N, dtype=int), demand_dist="poisson", mu=5, seed=1)
    return OracleEnv("IM_div", cfg, n_envs=1), OracleEnv("IM_div", cfg, n_envs=1, split="closed")


def test_oracle_closed_split_equals_literal_loops():
    """oracle/im_oracle.py's phase-at-a-time split (split="closed", used by the large-capacity GPU campaign)
    against the oracle's literal unit-by-unit loops on every (x, amt, guard) of a grid, 2-4 children, both
    loop kinds (backlog-first / outstanding orders with the sum check, the capped loop without), guard
    trips and spins included: counts, shipments, amount left and error flags identical."""
    import numpy as np
    rs = np.random.RandomState(5)
    for m in (2, 3, 4):
        lit, clo = _oracle_pair(m)
        n = 4000
        for env in (lit, clo):
            env.n = n
        x0 = rs.randint(-4, 14, size=(n, m)).astype(np.float64)
        amt0 = rs.randint(-2, 41, size=n).astype(np.float64)
        lim = rs.choice([0, 1, 2, 3, 5, 8, 60], size=n).astype(np.float64)
        active = rs.rand(n) < 0.9
        for kind in ("positive", "capped"):
            outs = []
            for env in (lit, clo):
                env.err = np.zeros(n, dtype=np.uint32)
                x, sto, amt = x0.copy(), np.zeros((n, m)), amt0.copy()
                if kind == "positive":
                    env._rr_positive(active, x, sto, amt, lim)
                    outs.append((x, sto, amt, env.err.copy()))
                else:
                    ordc = np.maximum(x0, 0).copy()      # order + backlog_to = x0: the cap as drawn
                    bto = x0 - ordc
                    env._rr_capped(active, bto, ordc, sto, amt, lim)
                    outs.append((sto, amt, env.err.copy()))
            for a, b in zip(*outs):
                np.testing.assert_array_equal(a, b, err_msg="%d children, %s loop" % (m, kind))
        assert outs[0][-1].any() and not outs[0][-1].all()      # guard trips occur on the grid


def test_oracle_closed_split_equals_literal_on_drawn_tree_episodes():
    """Whole episodes of drawn tree specifications (tests/fuzz_configs.py; small capacities, where the
    literal loop is fast) through both oracle split modes: every state, info and observation equal."""
    import numpy as np
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import test_fuzz_gpu as tf
    from oracle.im_oracle import OracleEnv
    checked = 0
    for i in range(2000, 2200):
        meta, d = tf.make_case(i)
        if not meta["kind"].endswith("div"):
            continue
        outs = []
        for split in ("literal", "closed"):
            env = OracleEnv(meta["kind"], meta["config"], n_envs=meta["E"], split=split)
            noisy = meta["noisy"]
            env.reset(customer_demand=d["customer_demand"], noisy_delay=bool(noisy), noisy_delay_threshold=noisy,
                      delay_uniforms=d["delay_uniforms"] if noisy else None)
            rec = []
            for t in range(meta["T"]):
                obs, rew, _, info = env.step(d["actions"][:, t, :])
                rec.append((obs, np.asarray(rew), info["ship_to"], info["backlog_to"], env.err.copy()))
            outs.append(rec)
        for a, b in zip(*outs):
            for u, v in zip(a, b):
                np.testing.assert_array_equal(u, v, err_msg="case %d" % i)
        checked += 1
        if checked == 12:
            break
    assert checked == 12

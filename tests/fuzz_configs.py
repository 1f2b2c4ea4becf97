"""Randomly drawn env configurations (test infrastructure): the generator behind
tests/golden/fuzz (tools/gen_fuzz_fixtures.py runs them through the reference), the exploratory
reference-vs-oracle run (tools/fuzz_explore.py) and the GPU-vs-oracle random-spec tests
(tests/test_fuzz_gpu.py). Configurations stay within what the reference's constructors accept.
"""
import numpy as np

def rand_tree(rs, N):
    """connections {parent: [children]} with child index > parent (utils.py:87-92), node 0 the
    factory, at most 3 children per node, every node reachable, and node N-1 at the deepest stage
    (the constructors take num_stages = get_stage(N - 1) + 1, IM_div_env.py:50)."""
    while True:
        conn = {i: [] for i in range(N)}
        depth = [0] * N
        for c in range(1, N):
            cands = [p for p in range(c) if len(conn[p]) < 3]
            p = cands[rs.randint(len(cands))]
            conn[p].append(c)
            depth[c] = depth[p] + 1
        if depth[N - 1] == max(depth):
            break
    for p in conn:
        if len(conn[p]) > 1 and rs.rand() < 0.3:     # child listing order is part of the split's order
            conn[p] = conn[p][::-1]
    return conn


SCALES = [30, 120, 5, 300, 40000]     # cycled by case index: every class meets every element width


def rand_config(rs, kind, idx):
    tree = kind in ("IM_div", "MAIM_div")
    N = rs.randint(3, 8) if tree else rs.randint(2, 9)
    T = int(rs.choice([10, 30, 50]))
    scale = SCALES[idx % len(SCALES)]
    inv_max = np.maximum(np.round(rs.uniform(0.5, 1.5, N) * scale), 2.0)
    init_inv = np.floor(rs.uniform(0, 1, N) * inv_max)
    c = dict(num_periods=T, init_inv=init_inv, inv_max=inv_max,
             inv_target=np.round(rs.uniform(0, 0.5, N) * inv_max),
             stock_cost=np.round(rs.uniform(0.05, 1.0, N), 2), backlog_cost=np.round(rs.uniform(0.1, 1.5, N), 2),
             delay=rs.randint(1, 6, N).astype(np.int8), demand_dist="custom", seed=int(rs.randint(1000)),
             time_dependency=bool(rs.rand() < 0.5), prev_demand=bool(rs.rand() < 0.5),
             prev_actions=bool(rs.rand() < 0.4), prev_length=int(rs.randint(1, 4)))
    if kind in ("MAIM", "MAIM_div") and c["prev_actions"] and not (c["prev_demand"] or c["time_dependency"]):
        c["prev_demand"] = True     # the reference's broken combination (MAIM_env.py:135-136) is rejected
    if tree:
        c.update(num_nodes=N, connections=rand_tree(rs, N))
        if kind == "IM_div":
            c["standardise_state"] = bool(rs.rand() < 0.8)
            c["standardise_actions"] = bool(rs.rand() < 0.8)
        else:
            c["share_network"] = bool(rs.rand() < 0.4)
            a = float(rs.choice([-1.0, 0.0, -2.0]))
            c.update(a=a, b=a + float(rs.choice([1.0, 2.0, 3.0])))
    else:
        c["num_stages"] = N
        c["price"] = np.cumsum(np.round(rs.uniform(0.5, 3.0, N + 1), 1))[::-1].copy()   # strictly decreasing
        c["standardise_state"] = bool(rs.rand() < 0.8)
        c["standardise_actions"] = bool(rs.rand() < 0.8)
        a = float(rs.choice([-1.0, 0.0, -2.0]))
        c.update(a=a, b=a + float(rs.choice([1.0, 2.0, 3.0])))
    if kind in ("MAIM", "MAIM_div"):
        c["independent"] = bool(rs.rand() < 0.4)
    return c


def maybe_order_max(rs, kind, c, p=0.3):
    """An explicit order_max (IM_env.py:55, IM_div_env.py:79) below or above the derived one, within
    the constructors' asserts (MAIM_env.py:171, MAIM_div_env.py:235)."""
    if rs.rand() >= p:
        return c
    N, im = len(c["inv_max"]), c["inv_max"]
    if "connections" in c:
        par = {ch: p_ for p_, chs in c["connections"].items() for ch in chs}
        om = np.array([im[0]] + [im[par[i]] for i in range(1, N)])
    else:
        om = np.array([im[i + 1] for i in range(N - 1)] + [im[N - 1]])
    om = np.maximum(np.floor(om * rs.uniform(0.3, 1.2, N)), 1.0)
    if kind == "MAIM":
        om[N - 1] = min(om[N - 1], im[N - 1])
    if kind == "MAIM_div":
        om[0] = min(om[0], im[0])
    c["order_max"] = om
    return c


def fuzz_inputs(kind, cfg, opts, seed, E=8):
    """Demand around each case's capacity scale; actions over [a, b] widened by 20 % (clipping), the
    exact bounds, and grid points that decode to half-integer orders (round-half-even)."""
    rs = np.random.RandomState(seed)
    N = cfg.get("num_stages", cfg.get("num_nodes"))
    T = cfg["num_periods"]
    R = sum(1 for v in cfg["connections"].values() if not v) if "connections" in cfg else 1
    top = float(np.max(cfg["inv_max"]))
    mus = top * np.array([0.05, 0.2, 0.5, 1.0])[rs.randint(0, 4, size=E)]
    dem = rs.poisson(mus[:, None, None], size=(E, R, T)).astype(np.int64)
    std_act = cfg.get("standardise_actions", True) or kind == "MAIM_div"
    if std_act:
        a = cfg.get("a", -1.0) if kind != "IM_div" else -1.0
        b = cfg.get("b", 1.0) if kind != "IM_div" else 1.0
        w = b - a
        act = rs.uniform(a - 0.2 * w, b + 0.2 * w, size=(E, T, N))
        act[0] = a
        act[1] = b
        act[2] = a + w * (rs.randint(0, 61, size=(T, N)) / 60.0)
    else:
        act = rs.uniform(-0.1 * top, 1.2 * top, size=(E, T, N))
        act[0] = 0.0
        act[1] = np.round(rs.uniform(0, top, size=(T, N))) + 0.5
    unif = rs.uniform(0, 1, size=(E, T, N))
    return dem, act, unif



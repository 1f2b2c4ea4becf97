"""EnvSpec: one frozen description of an env batch, derived from a reference config dict.

``build_spec(kind, config)`` restates the constructor of the matching reference
class — the defaults, the derived capacities and prices, and every per-class
difference in observation scaling, order decoding, backlog capping and reward
aggregation — into flat per-node vectors (``HostSpec``) that the HIP step kernel
consumes through the C ABI (``ImEnvSpec`` in include/imenv.h).

  kind "IM"        InvManagement.__init__              environments/IM_env.py:7-162
  kind "MAIM"      MultiAgentInvManagement.__init__    environments/MAIM_env.py:8-173
  kind "IM_div"    InvManagementDiv.__init__           environments/IM_div_env.py:9-199
  kind "MAIM_div"  MultiAgentInvManagementDiv.__init__ environments/MAIM_div_env.py:9-237

Constraints of this build (raise ValueError, documented in DESIGN.md): capacities,
initial inventory and delays must be integral (the reference stores them as
float64 but every config in the repo is integral); delay >= 1; N <= 16 nodes;
<= 8 children per node; prev_length <= 8.
"""
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from . import _native as nat
from .topology import check_connections, create_network, get_retailers, get_stage

KINDS = ("IM", "MAIM", "IM_div", "MAIM_div")


class SpecError(ValueError):
    pass


def _vec(x, n, dtype=np.float64):
    v = np.asarray(x, dtype=np.float64).reshape(-1)
    if v.shape[0] != n:
        raise SpecError("expected %d values, got %d" % (n, v.shape[0]))
    return v.astype(dtype)


def _integral(name, v):
    v = np.asarray(v, dtype=np.float64)
    if not np.all(np.isfinite(v)) or not np.all(v == np.round(v)):
        raise SpecError("%s must be integral in this build (got %s)" % (name, v.tolist()))
    return v.astype(np.int64)


@dataclass
class HostSpec:
    """Host mirror of a spec: what the adaptors and callers read (env.order_max, env.a, ...)."""
    kind: str
    num_nodes: int
    num_periods: int
    parent: np.ndarray
    children: List[List[int]]
    retailers: List[int]
    delay: np.ndarray
    init_inv: np.ndarray
    inv_max: np.ndarray
    order_max: np.ndarray
    demand_max: Optional[np.ndarray]
    backlog_cap: np.ndarray
    sell_price: np.ndarray
    buy_price: np.ndarray
    stock_cost: np.ndarray
    backlog_cost: np.ndarray
    inv_target: np.ndarray
    a: float
    b: float
    standardise_state: bool
    standardise_actions: bool
    time_dependency: bool
    prev_demand: bool
    prev_actions: bool
    prev_length: int
    max_delay: int
    independent: bool
    share_network: bool
    features: List[tuple]          # (group, index)
    group_mode: Dict[int, int]
    group_den: Dict[int, np.ndarray]
    group_clip: Dict[int, np.ndarray]
    decode_mode: int
    reward_mode: int
    demand_dist: str
    mu: float
    lower_upper: tuple
    custom_demand: Optional[np.ndarray]
    noisy_demand: bool
    noisy_demand_threshold: float
    noisy_delay: bool
    noisy_delay_threshold: float
    seed: int
    split_limit: np.ndarray
    connections: Optional[dict] = None
    config: dict = field(default_factory=dict)

    @property
    def num_features(self):
        return len(self.features)

    @property
    def num_retailers(self):
        return len(self.retailers)

    @property
    def multi_agent(self):
        return self.kind in ("MAIM", "MAIM_div")

    @property
    def serial(self):
        return self.kind in ("IM", "MAIM")

    def to_c(self):
        N = self.num_nodes
        s = nat.ImEnvSpec()
        s.abi_version = nat.ABI_VERSION
        s.kind = nat.KIND[self.kind]
        s.num_nodes = N
        s.num_periods = self.num_periods
        for i in range(nat.MAXN):
            s.parent[i] = -1
            s.demand_parent[i] = -1
            s.retailer_slot[i] = -1
            s.backlog_cap[i] = -1
        for i in range(N):
            s.parent[i] = int(self.parent[i])
            s.num_children[i] = len(self.children[i])
            for k, c in enumerate(self.children[i]):
                s.children[i][k] = int(c)
            s.delay[i] = int(self.delay[i])
            s.init_inv[i] = int(self.init_inv[i])
            s.inv_max[i] = int(self.inv_max[i])
            s.order_max[i] = int(self.order_max[i])
            s.backlog_cap[i] = int(self.backlog_cap[i])
            for q in range(4):
                s.split_limit[i][q] = int(self.split_limit[i][q])
            s.sell_price[i] = float(self.sell_price[i])
            s.buy_price[i] = float(self.buy_price[i])
            s.stock_cost[i] = float(self.stock_cost[i])
            s.backlog_cost[i] = float(self.backlog_cost[i])
            s.inv_target[i] = float(self.inv_target[i])
        for c in range(N):
            p = int(self.parent[c])
            if p >= 0 and (self.serial or c >= p):     # IM_div_env.py:385 scans j >= i
                s.demand_parent[c] = p
        for k, r in enumerate(self.retailers):
            s.retailer_slot[r] = k
        s.num_retailers = len(self.retailers)
        s.standardise_actions = int(self.standardise_actions)
        s.decode_mode = self.decode_mode
        s.a = float(self.a)
        s.b = float(self.b)
        s.reward_mode = self.reward_mode
        s.num_features = len(self.features)
        for f, (g, j) in enumerate(self.features):
            s.feat_group[f] = g
            s.feat_index[f] = j
        for g in range(nat.NGROUPS):
            s.group_mode[g] = self.group_mode.get(g, nat.OBS_ZERO)
            den = self.group_den.get(g)
            clip = self.group_clip.get(g)
            for i in range(N):
                s.group_den[g][i] = float(den[i]) if den is not None else 1.0
                s.group_clip[g][i] = float(clip[i]) if clip is not None else float("inf")
        s.prev_length = self.prev_length
        s.demand_dist = {"custom": nat.DEMAND_CUSTOM, "poisson": nat.DEMAND_POISSON,
                         "uniform": nat.DEMAND_UNIFORM}[self.demand_dist]
        s.poisson_mu = float(self.mu)
        s.uniform_low, s.uniform_high = int(self.lower_upper[0]), int(self.lower_upper[1])
        s.noisy_demand = int(self.noisy_demand)
        s.noisy_demand_threshold = float(self.noisy_demand_threshold)
        s.noisy_delay = int(self.noisy_delay)
        s.noisy_delay_threshold = float(self.noisy_delay_threshold)
        s.seed = int(self.seed) & 0xFFFFFFFFFFFFFFFF
        return s


def build_spec(kind, config, num_periods=None):
    """Derive a HostSpec from a reference-style env_config dict (not mutated)."""
    if kind not in KINDS:
        raise SpecError("unknown env kind %r" % (kind,))
    cfg = dict(config)
    if num_periods is not None:
        cfg["num_periods"] = num_periods
    if kind in ("IM", "MAIM"):
        return _serial(kind, cfg)
    return _tree(kind, cfg)


def _common_tail(kind, g, N):
    td = bool(g("time_dependency", False))
    pa = bool(g("prev_actions", False))
    pd = bool(g("prev_demand", False))
    L = int(g("prev_length", 1))
    if L < 1 or L > 8:
        raise SpecError("prev_length must be in 1..8 in this build")
    return td, pa, pd, L


def _demand_params(g, R, T, serial=False):
    dist = g("demand_dist", "custom")
    if dist not in ("custom", "poisson", "uniform"):
        raise SpecError("Unrecognised, Distribution Not Implemented")   # IM_env.py:206-207
    mu = float(g("mu", 5))
    lu = tuple(g("lower_upper", (1, 5)))
    if dist == "uniform" and lu[0] >= lu[1]:
        raise SpecError("Lower bound cannot be larger than upper bound")  # IM_env.py:203-204
    custom = None
    if dist == "custom":
        cd = g("customer_demand", None)
        if cd is None:                               # IM_env.py:189 ([T]) / IM_div_env.py:226 ([R, T])
            cd = np.ones(T) * 5 if serial else np.ones((R, T)) * 5
        custom = np.asarray(cd)
    return dist, mu, lu, custom


def _serial(kind, cfg):
    g = cfg.get
    ma = kind == "MAIM"
    T = int(g("num_periods", 50))
    N = int(g("num_stages", 3))
    if N < 1 or N > nat.MAXN:
        raise SpecError("num_stages must be in 1..%d" % nat.MAXN)
    init_inv = _integral("init_inv", _vec(g("init_inv", np.ones(N) * (100 if ma else 20)), N))
    delay = _integral("delay", _vec(g("delay", np.ones(N)), N))
    std_s = bool(g("standardise_state", True))
    std_a = bool(g("standardise_actions", True))
    a = g("a", -1)
    b = g("b", 1)
    td, pa, pd, L = _common_tail(kind, g, N)
    D = int(delay.max())
    if D == 0:
        td = False                                   # IM_env.py:27-29
    price = _vec(g("price", np.flip(np.arange(N + 1) + 1)), N + 1)
    inv_target = _vec(g("inv_target", np.ones(N) * 10), N)
    stock_cost = _vec(g("stock_cost", np.ones(N) * 0.5), N)
    backlog_cost = _vec(g("backlog_cost", np.ones(N)), N)
    inv_max = _integral("inv_max", _vec(g("inv_max", np.ones(N) * (200 if ma else 100)), N))
    om = np.zeros(N)
    for i in range(N - 1):                           # IM_env.py:51-54
        om[i] = inv_max[i + 1]
    om[N - 1] = inv_max[N - 1]
    order_max = _integral("order_max", _vec(g("order_max", om), N))
    if ma:
        # MAIM_env.py:158-171 runtime checks
        if not isinstance(T, int):
            raise SpecError("num_periods must be an int")
        for i in range(len(price) - 1):
            if not price[i] > price[i + 1]:
                raise SpecError("sell price of a stage must exceed its upstream stage's (MAIM_env.py:167-168)")
        if not order_max[N - 1] <= inv_max[N - 1]:
            raise SpecError("order_max of the last stage cannot exceed its inventory (MAIM_env.py:171)")
        if pa and not pd and not td:
            raise SpecError("Not Implemented (MAIM_env.py:135-136: prev_actions without prev_demand)")
    imf = inv_max.astype(np.float64)
    omf = order_max.astype(np.float64)
    feats, mode, den, clip = [(nat.G_INV, 0), (nat.G_BACKLOG, 0), (nat.G_ORDER_U, 0)], {}, {}, {}
    if kind == "IM":
        # IM_env.py:231-285: base scaled iff standardise_state; history ALWAYS scaled; tds iff std
        for gg, dd in ((nat.G_INV, imf), (nat.G_BACKLOG, imf), (nat.G_ORDER_U, imf)):
            mode[gg] = nat.OBS_SCALED if std_s else nat.OBS_RAW
            den[gg] = dd
        mode[nat.G_DEMAND_HIST], den[nat.G_DEMAND_HIST] = nat.OBS_SCALED, imf
        mode[nat.G_ORDER_HIST], den[nat.G_ORDER_HIST] = nat.OBS_SCALED, omf
        mode[nat.G_TRANSIT], den[nat.G_TRANSIT] = (nat.OBS_SCALED if std_s else nat.OBS_RAW), imf
        feats += _tail_feats(pd, pa, td, L, D)
    else:
        if std_s:
            # MAIM_env.py:296-317: order_u scaled by order_max
            for gg, dd in ((nat.G_INV, imf), (nat.G_BACKLOG, imf), (nat.G_ORDER_U, omf)):
                mode[gg], den[gg] = nat.OBS_SCALED, dd
            mode[nat.G_DEMAND_HIST], den[nat.G_DEMAND_HIST] = nat.OBS_SCALED, imf
            mode[nat.G_ORDER_HIST], den[nat.G_ORDER_HIST] = nat.OBS_SCALED, omf
            mode[nat.G_TRANSIT], den[nat.G_TRANSIT] = nat.OBS_SCALED, imf
            if pd and not pa and not td:
                # MAIM_env.py:296-317 has no branch for prev_demand alone: its L slots stay 0
                feats += [(nat.G_ZERO, 0)] * L
            else:
                feats += _tail_feats(pd, pa, td, L, D)
        else:
            # MAIM_env.py:319-324: raw base; raw tds in slots 3..3+D-1; every other slot stays 0
            for gg in (nat.G_INV, nat.G_BACKLOG, nat.G_ORDER_U, nat.G_TRANSIT):
                mode[gg] = nat.OBS_RAW
            F = 3 + L * int(pd) + L * int(pa) + D * int(td)
            tail = [(nat.G_TRANSIT, k) for k in range(D)] if td else []
            tail += [(nat.G_ZERO, 0)] * (F - 3 - len(tail))
            feats += tail
    dist, mu, lu, custom = _demand_params(g, 1, T, serial=True)
    return HostSpec(
        kind=kind, num_nodes=N, num_periods=T,
        parent=np.array([i + 1 for i in range(N - 1)] + [-1]),
        children=[[i - 1] if i > 0 else [] for i in range(N)], retailers=[0],
        delay=delay, init_inv=init_inv, inv_max=inv_max, order_max=order_max, demand_max=None,
        backlog_cap=inv_max.copy() if std_s else np.full(N, -1),   # IM_env.py:319-320
        sell_price=price[0:N].copy(), buy_price=price[1:N + 1].copy(),   # IM_env.py:365
        stock_cost=stock_cost, backlog_cost=backlog_cost, inv_target=inv_target,
        a=a, b=b, standardise_state=std_s, standardise_actions=std_a,
        time_dependency=td, prev_demand=pd, prev_actions=pa, prev_length=L, max_delay=D,
        independent=bool(g("independent", True)) if ma else False, share_network=False,
        features=feats, group_mode=mode, group_den=den, group_clip=clip,
        decode_mode=nat.DECODE_ROUND_CLIP if ma else nat.DECODE_CLIP_ROUND,
        reward_mode=(nat.REWARD_INDEPENDENT if bool(g("independent", True)) else nat.REWARD_SHARED_MEAN)
        if ma else nat.REWARD_SUM,
        demand_dist=dist, mu=mu, lower_upper=lu, custom_demand=custom,
        noisy_demand=False, noisy_demand_threshold=0.0, noisy_delay=False, noisy_delay_threshold=0.0,
        seed=int(g("seed", 52)), split_limit=np.zeros((N, 4), dtype=np.int64), config=cfg)


def _tail_feats(pd, pa, td, L, D, share=False):
    f = []
    if pd:
        f += [(nat.G_DEMAND_HIST, j) for j in range(L)]
    if pa:
        f += [(nat.G_ORDER_HIST, j) for j in range(L)]
    if td:
        f += [(nat.G_TRANSIT, k) for k in range(D)]
    if share:
        f += [(nat.G_NODE_ID, 0)]
    return f


def _tree(kind, cfg):
    g = cfg.get
    ma = kind == "MAIM_div"
    T = int(g("num_periods", 50))
    N = int(g("num_nodes", 3))
    conn = g("connections", {0: [1], 1: [2], 2: []})
    conn = {int(k): [int(c) for c in (v or [])] for k, v in conn.items()}
    check_connections(conn)
    net = create_network(conn)
    if net.shape[0] != N:
        raise SpecError("connections describe %d nodes, num_nodes is %d" % (net.shape[0], N))
    if N > nat.MAXN:
        raise SpecError("num_nodes must be <= %d" % nat.MAXN)
    retailers = get_retailers(net)
    parent = np.full(N, -1)
    for i in range(1, N):                            # IM_div_env.py:26-28
        ups = np.where(net.T[i] == 1)[0]
        if len(ups) != 1:
            raise SpecError("node %d needs exactly one upstream node" % i)
        parent[i] = int(ups[0])
    if any(parent[i] < 0 for i in range(1, N)):
        raise SpecError("only node 0 may be the factory")
    children = [list(conn.get(i, [])) for i in range(N)]
    if max(len(c) for c in children) > nat.MAXC:
        raise SpecError("at most %d children per node in this build" % nat.MAXC)
    num_stages = get_stage(N - 1, net) + 1
    init_inv = _integral("init_inv", _vec(g("init_inv", np.ones(N) * (100 if ma else 20)), N))
    delay = _integral("delay", _vec(g("delay", np.ones(N)), N))
    std_s = True if ma else bool(g("standardise_state", True))
    std_a = True if ma else bool(g("standardise_actions", True))
    a = g("a", -1) if ma else -1                     # IM_div_env.py:35-36 hard-codes the interval
    b = g("b", 1) if ma else 1
    td, pa, pd, L = _common_tail(kind, g, N)
    D = int(delay.max())
    if D == 0:
        td = False
    share = bool(g("share_network", False)) if ma else False
    if ma and pa and not pd and not td:
        raise SpecError("Not Implemented (MAIM_div_env.py:164-165,218-219)")
    stage_price = np.arange(num_stages) + 2          # IM_div_env.py:54-60
    stage_cost = np.arange(num_stages) + 1
    sell = np.array([stage_price[get_stage(i, net)] for i in range(N)], dtype=np.float64)
    buy = np.array([stage_cost[get_stage(i, net)] for i in range(N)], dtype=np.float64)
    inv_target = _vec(g("inv_target", np.ones(N) * (0 if ma else 10)), N)
    stock_cost = _vec(g("stock_cost", np.ones(N) * 0.5), N)
    backlog_cost = _vec(g("backlog_cost", np.ones(N)), N)
    inv_max = _integral("inv_max", _vec(g("inv_max", np.ones(N) * 100), N))
    om = np.zeros(N)
    for i in range(1, N):                            # IM_div_env.py:75-78
        om[i] = inv_max[parent[i]]
    om[0] = inv_max[0]
    order_max = _integral("order_max", _vec(g("order_max", om), N))
    if ma and not order_max[0] <= inv_max[0]:
        raise SpecError("order_max of node 0 cannot exceed its inventory (MAIM_div_env.py:235)")
    dm = inv_max.copy()                              # IM_div_env.py:83-92
    for i in range(N):
        s = int(sum(order_max[j] for j in range(N) if net[i][j] == 1))
        if s > dm[i]:
            dm[i] = s
    imf, omf, dmf = inv_max.astype(float), order_max.astype(float), dm.astype(float)
    feats, mode, den, clip = [(nat.G_INV, 0), (nat.G_BACKLOG, 0), (nat.G_ORDER_U, 0)], {}, {}, {}
    if kind == "IM_div":
        # IM_div_env.py:304-359: backlog / demand history scaled by demand_max
        for gg, dd in ((nat.G_INV, imf), (nat.G_BACKLOG, dmf), (nat.G_ORDER_U, imf)):
            mode[gg], den[gg] = (nat.OBS_SCALED if std_s else nat.OBS_RAW), dd
        mode[nat.G_DEMAND_HIST], den[nat.G_DEMAND_HIST] = nat.OBS_SCALED, dmf
        mode[nat.G_ORDER_HIST], den[nat.G_ORDER_HIST] = nat.OBS_SCALED, omf
        mode[nat.G_TRANSIT], den[nat.G_TRANSIT] = (nat.OBS_SCALED if std_s else nat.OBS_RAW), imf
    else:
        # MAIM_div_env.py:387-435
        for gg, dd in ((nat.G_INV, imf), (nat.G_BACKLOG, dmf), (nat.G_ORDER_U, omf)):
            mode[gg], den[gg] = nat.OBS_SCALED, dd
        mode[nat.G_DEMAND_HIST], den[nat.G_DEMAND_HIST] = nat.OBS_SCALED, dmf
        mode[nat.G_ORDER_HIST], den[nat.G_ORDER_HIST] = nat.OBS_SCALED, omf
        mode[nat.G_TRANSIT], den[nat.G_TRANSIT] = nat.OBS_CLAMP_SCALED, imf * 2
        clip[nat.G_TRANSIT] = imf * 2
        mode[nat.G_NODE_ID], den[nat.G_NODE_ID] = nat.OBS_SCALED, np.full(N, float(N))
    if ma and pd and not pa and not td:
        # MAIM_div_env.py:413-432 has no branch for prev_demand alone: its L slots stay 0
        feats += [(nat.G_ZERO, 0)] * L + ([(nat.G_NODE_ID, 0)] if share else [])
    else:
        feats += _tail_feats(pd, pa, td, L, D, share)
    R = len(retailers)
    dist, mu, lu, custom = _demand_params(g, R, T)
    # guard limits: IM_div x(4,2,2,2), MAIM_div x(2,1,1,1) of demand_max (IM_div_env.py:424-497)
    mult = (2, 1, 1, 1) if ma else (4, 2, 2, 2)
    split_limit = np.array([[int(dm[i]) * m for m in mult] for i in range(N)], dtype=np.int64)
    ind = bool(g("independent", True)) if ma else False
    return HostSpec(
        kind=kind, num_nodes=N, num_periods=T, parent=parent, children=children, retailers=retailers,
        delay=delay, init_inv=init_inv, inv_max=inv_max, order_max=order_max, demand_max=dm,
        backlog_cap=dm.copy() if (ma or std_s) else np.full(N, -1),   # IM_div_env.py:508, MAIM_div:584
        sell_price=sell, buy_price=buy, stock_cost=stock_cost, backlog_cost=backlog_cost,
        inv_target=inv_target, a=a, b=b, standardise_state=std_s, standardise_actions=std_a,
        time_dependency=td, prev_demand=pd, prev_actions=pa, prev_length=L, max_delay=D,
        independent=ind, share_network=share, features=feats, group_mode=mode, group_den=den,
        group_clip=clip, decode_mode=nat.DECODE_ROUND_CLIP if ma else nat.DECODE_CLIP_ROUND,
        reward_mode=(nat.REWARD_INDEPENDENT if ind else nat.REWARD_SHARED_MEAN) if ma else nat.REWARD_SUM,
        demand_dist=dist, mu=mu, lower_upper=lu, custom_demand=custom,
        noisy_demand=bool(g("noisy_demand", False)),
        noisy_demand_threshold=float(g("noisy_demand_threshold", 0)),
        noisy_delay=bool(g("noisy_delay", False)), noisy_delay_threshold=float(g("noisy_delay_threshold", 0)),
        seed=int(g("seed", 52)), split_limit=split_limit, connections=conn, config=cfg)

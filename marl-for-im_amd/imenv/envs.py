"""Drop-in adaptors: the reference's four env classes, same constructor, attributes and methods,
with the dynamics running in the HIP step kernel.

    from imenv.envs import InvManagement, MultiAgentInvManagement, InvManagementDiv, \\
        MultiAgentInvManagementDiv
    env = MultiAgentInvManagement(config)          # == environments/MAIM_env.py:MultiAgentInvManagement
    obs = env.reset()
    obs, rewards, dones, infos = env.step({"stage_0": [0.3], ...})

Each adaptor is one env (n_envs = 1 of VectorInvEnv, float64 observations) and re-exposes what the
reference's callers read: observation_space / action_space, num_agents, agent ids
stage_i / node_i, "__all__", the info keys (period, demand, ship, acquisition, profit,
'actual order'), the history arrays inv / backlog / order_u / demand / ship / acquisition / order_r
indexed by period (base_restock_policy.py:12), order_max / inv_max / a / b / dist / dist_param /
customer_demand, and rescale / rev_scale.

Host randomness follows the reference exactly, so a seeded adaptor reproduces the reference's own
trajectories: np.random.seed(seed) in the constructor (IM_env.py:46), demand drawn at reset with
scipy's poisson / randint on NumPy's global stream (IM_env.py:186-205), the div envs' noisy demand
drawn on the host in the reference's order (IM_div_env.py:246-255), and noisy-delay uniforms drawn
at each step, factory first, one per node with t - d >= 0 (IM_env.py:384-407), then handed to the
kernel (imenv_set_delay_uniforms). The reference's quirks are kept: IM / MAIM pop their keys from
the caller's config dict and pop mu / customer_demand / lower_upper from their own copy at the first
reset (later resets fall back to the defaults); the constructor calls reset() once.

For throughput use VectorInvEnv directly (batched, device tensors, in-kernel Philox demand).
"""
import numpy as np
import torch
from scipy.stats import poisson, randint

from . import _native as nat
from .spaces import Box
from .spec import build_spec
from .vector_env import VectorInvEnv

try:  # pragma: no cover - base classes only where the frameworks are installed
    import gym
    _GymEnv = gym.Env
except Exception:
    _GymEnv = object
try:  # pragma: no cover
    from ray.rllib.env.multi_agent_env import MultiAgentEnv as _MultiAgentEnv
except Exception:
    _MultiAgentEnv = object

# keys the serial constructors pop from the CALLER's dict (IM_env.py:11-55, MAIM_env.py:13-62)
_SERIAL_POPS = {
    "IM": ("num_periods", "num_stages", "init_inv", "delay", "standardise_state", "standardise_actions", "a", "b",
           "time_dependency", "prev_actions", "prev_demand", "prev_length", "price", "inv_target", "stock_cost",
           "backlog_cost", "demand_dist", "seed", "inv_max", "order_max"),
    "MAIM": ("num_periods", "independent", "num_stages", "standardise_state", "standardise_actions", "a", "b",
             "num_agents", "init_inv", "inv_target", "delay", "time_dependency", "prev_actions", "prev_demand",
             "prev_length", "price", "stock_cost", "backlog_cost", "demand_dist", "seed", "inv_max", "order_max"),
}


def rescale(val, min_val, max_val, A=-1, B=1):
    """IM_env.py:435-444."""
    return A + ((val - min_val) * (B - A)) / (max_val - min_val)


def rev_scale(val_scaled, min_val, max_val, A=-1, B=1):
    """IM_env.py:446-456."""
    return ((val_scaled - A) * (max_val - min_val)) / (B - A) + min_val


def make_spaces(kind, sp):
    """(observation_space, action_space) of ONE env of the reference class `kind` (per agent for the
    multi-agent classes): IM_env.py:60-139, MAIM_env.py:67-153, IM_div_env.py:95-180,
    MAIM_div_env.py:103-218."""
    N, F = sp.num_nodes, sp.num_features
    ma = sp.multi_agent
    a, b = sp.a, sp.b
    inv_max = np.asarray(sp.inv_max, dtype=np.float64)
    order_max = np.asarray(sp.order_max, dtype=np.float64)
    obs_shape = (F,) if ma else (N, F)
    if sp.standardise_state or kind == "MAIM_div":
        obs_space = Box(low=np.ones(obs_shape) * a, high=np.ones(obs_shape) * b, dtype=np.float64, shape=obs_shape)
    else:
        # raw observations (IM_env.py:129-139, MAIM_env.py:138-153): inv, backlog (unbounded), order_u,
        # then in-transit slots, all bounded by the largest capacity
        m = float(np.max(inv_max))
        high = np.full(obs_shape, m)
        high[..., 1] = np.inf
        obs_space = Box(low=np.zeros(obs_shape), high=high, dtype=np.float64, shape=obs_shape)
    act_n = 1 if ma else N
    if sp.standardise_actions or kind == "MAIM_div":
        act_space = Box(low=np.ones(act_n) * a, high=np.ones(act_n) * b, dtype=np.float64, shape=(act_n,))
    else:
        high = np.ones(1) * np.max(order_max) if ma else order_max
        act_space = Box(low=np.zeros(act_n), high=high, dtype=np.int32, shape=(act_n,))
    return obs_space, act_space


class _Adaptor:
    KIND = None

    def __init__(self, config, device=None):
        self.config = config.copy()
        self.spec = sp = build_spec(self.KIND, config)
        for k in _SERIAL_POPS.get(self.KIND, ()):
            config.pop(k, None)
        N, T = sp.num_nodes, sp.num_periods
        self.num_periods = T
        self.num_nodes = N
        self.serial = sp.serial
        if sp.serial:
            self.num_stages = N
        else:
            self.connections = sp.connections
            self.retailers = list(sp.retailers)
            self.non_retailers = [i for i in range(N) if i not in self.retailers]
            self.upstream_node = {i: int(sp.parent[i]) for i in range(1, N)}
            self.num_stages = int(self.config.get("_num_stages", 0)) or self._tree_depth()
            self.demand_max = sp.demand_max.astype(np.float64)
            self.node_price = sp.sell_price.copy()
            self.node_cost = sp.buy_price.copy()
        self.inv_init = sp.init_inv.astype(np.float64)
        self.delay = np.asarray(sp.delay)
        self.max_delay = int(sp.max_delay)
        self.inv_max = sp.inv_max.astype(np.float64)
        self.order_max = sp.order_max.astype(np.float64)
        self.inv_target = sp.inv_target
        self.stock_cost = sp.stock_cost
        self.backlog_cost = sp.backlog_cost
        if sp.serial:
            self.price = np.concatenate([sp.sell_price, sp.buy_price[-1:]])
        self.a, self.b = sp.a, sp.b
        self.standardise_state = sp.standardise_state
        self.standardise_actions = sp.standardise_actions
        self.time_dependency = sp.time_dependency
        self.prev_actions = sp.prev_actions
        self.prev_demand = sp.prev_demand
        self.prev_length = sp.prev_length
        self.demand_dist = sp.demand_dist
        self.noisy_demand = sp.noisy_demand
        self.noisy_demand_threshold = sp.noisy_demand_threshold
        self.noisy_delay = sp.noisy_delay                 # div envs read it from config (IM_div_env.py:50-51)
        self.noisy_delay_threshold = sp.noisy_delay_threshold
        self.SEED = sp.seed
        self.done = set()
        np.random.seed(seed=int(self.SEED))              # IM_env.py:46: the process-global stream
        self._setup_spaces()
        self._env = VectorInvEnv(sp, n_envs=1, device=device, obs_dtype=torch.float64)
        self._step_buffers()
        self._uniform_order = ([N - 1] + list(range(N - 1))) if sp.serial else list(range(N))
        self.period = 0
        self.reset()

    # ------------------------------------------------------------------ construction helpers
    def _step_buffers(self):
        """Persistent buffers of the per-step round trip: everything step() returns is written by the
        kernels into two device buffers (float64: obs | reward | profit; int32: order, demand,
        acquisition, ship, ship_to, backlog_to, inv, backlog, order_u, split-guard flag), copied to
        pinned host memory with two asynchronous copies and one synchronisation per step."""
        N, F = self.num_nodes, self.spec.num_features
        nr = N if self.spec.reward_mode == nat.REWARD_INDEPENDENT else 1
        dev = self._env.device
        self._dev_f = torch.empty(N * F + nr + N, dtype=torch.float64, device=dev)
        self._dev_i = torch.empty(9 * N + 1, dtype=torch.int32, device=dev)
        self._host_f = torch.empty(self._dev_f.shape, dtype=torch.float64, pin_memory=True)
        self._host_i = torch.empty(self._dev_i.shape, dtype=torch.int32, pin_memory=True)
        self._host_a = torch.empty((1, N), dtype=torch.float64, pin_memory=True)
        self._dev_a = torch.empty((1, N), dtype=torch.float64, device=dev)
        f, i = self._dev_f, self._dev_i
        self._obs_v = f[:N * F].view(1, N, F)
        self._rew_v = f[N * F:N * F + nr].view((1, N) if nr == N else (1,))
        iv = lambda j: i[j * N:(j + 1) * N].view(1, N)
        self._info_v = dict(order=iv(0), demand=iv(1), acquisition=iv(2), ship=iv(3),
                            profit=f[N * F + nr:].view(1, N), ship_to=iv(4), backlog_to=iv(5))
        self._state_v = [i[(6 + j) * N:(7 + j) * N].view(N, 1) for j in range(3)]
        self._flag_v = i[9 * N:]
        self._nr = nr

    def _tree_depth(self):
        depth = np.zeros(self.num_nodes, dtype=int)
        for i in range(1, self.num_nodes):
            depth[i] = depth[self.upstream_node[i]] + 1
        return int(depth.max()) + 1

    def _setup_spaces(self):
        self.observation_space, self.action_space = make_spaces(self.KIND, self.spec)

    # ------------------------------------------------------------------ reference helpers
    def rescale(self, val, min_val, max_val, A=-1, B=1):
        return rescale(val, min_val, max_val, A, B)

    def rev_scale(self, val_scaled, min_val, max_val, A=-1, B=1):
        return rev_scale(val_scaled, min_val, max_val, A, B)

    # ------------------------------------------------------------------ demand (host, reference RNG)
    def _draw_demand(self):
        R, T = len(self.spec.retailers), self.num_periods
        size = T if self.serial else (R, T)
        get = self.config.pop if self.serial else self.config.get     # IM_env.py:189 vs IM_div_env.py:226
        if self.demand_dist == "custom":
            default = np.ones(T, dtype=np.int16) * 5 if self.serial else np.ones((R, T), dtype=np.int16) * 5
            cd = get("customer_demand", default)
        elif self.demand_dist == "poisson":
            self.mu = get("mu", 5)
            self.dist = poisson
            self.dist_param = {"mu": self.mu}
            cd = self.dist.rvs(size=size, **self.dist_param)
        elif self.demand_dist == "uniform":
            lower, upper = get("lower_upper", (1, 5))[:2]
            self.dist = randint
            self.dist_param = {"low": lower, "high": upper}
            if lower >= upper:
                raise Exception("Lower bound cannot be larger than upper bound")
            cd = self.dist.rvs(size=size, **self.dist_param)
        else:
            raise Exception("Unrecognised, Distribution Not Implemented")
        if not self.serial and self.noisy_demand:       # IM_div_env.py:246-255, in place like the reference
            for k in range(R):
                for j in range(T):
                    double_demand = np.random.uniform(0, 1)
                    zero_demand = np.random.uniform(0, 1)
                    if double_demand <= self.noisy_demand_threshold:
                        cd[k, j] = 2 * cd[k, j]
                    if zero_demand <= self.noisy_demand_threshold:
                        cd[k, j] = 0
        return cd

    # ------------------------------------------------------------------ API
    def reset(self, customer_demand=None, noisy_delay=False, noisy_delay_threshold=0):
        """IM_env.py:164-229 (and siblings)."""
        T, N = self.num_periods, self.num_nodes
        if noisy_delay:
            self.noisy_delay = noisy_delay
            self.noisy_delay_threshold = noisy_delay_threshold
        self.customer_demand = customer_demand if customer_demand is not None else self._draw_demand()
        cd = np.asarray(self.customer_demand)
        table = cd.reshape(1, T) if self.serial else cd.reshape(1, cd.shape[0], -1)
        self.inv = np.zeros([T + 1, N])
        self.order_r = np.zeros([T, N])
        self.order_u = np.zeros([T + 1, N])
        self.ship = np.zeros([T, N])
        self.acquisition = np.zeros([T, N])
        self.backlog = np.zeros([T + 1, N])
        self.demand = np.zeros([T + 1, N])
        self.period = 0
        for r, node in enumerate(self.spec.retailers):
            self.demand[0, node] = (cd[0] if self.serial else cd[r, 0])
        self.inv[0, :] = self.inv_init
        obs = self._env.reset(customer_demand=table[..., :T], noisy_delay=bool(self.noisy_delay),
                              noisy_delay_threshold=float(self.noisy_delay_threshold))
        self.state = self._wrap_obs(obs.cpu().numpy()[0])
        return self.state

    def _actions(self, action):
        raise NotImplementedError

    def step(self, action):
        """IM_env.py:287-360 (and siblings)."""
        t, N = self.period, self.num_nodes
        if t >= self.num_periods:
            raise IndexError("index %d is out of bounds for axis 0 with size %d" % (t, self.num_periods))
        act = self._actions(action)
        if self.noisy_delay:       # one uniform per node with t - d >= 0, factory first (IM_env.py:384-407)
            u = np.ones(N)
            for i in self._uniform_order:
                if t - int(self.delay[i]) >= 0:
                    u[i] = np.random.uniform(0, 1)
            self._env.set_delay_uniforms(t, u[None, :])
        self._host_a.numpy()[0] = act                 # pinned; the previous step's copies have completed
        self._dev_a.copy_(self._host_a, non_blocking=True)
        env = self._env
        env.step(self._dev_a, obs_out=self._obs_v, reward_out=self._rew_v, info_out=self._info_v)
        env.state(out=self._state_v)
        if not self.serial:    # per-env split-guard flag into the int32 buffer (no separate round trip)
            nat.check(env.lib.imenv_get_errors(env._h, self._flag_v.data_ptr(), None, env._stream()),
                      "imenv_get_errors")
        self._host_f.copy_(self._dev_f, non_blocking=True)
        self._host_i.copy_(self._dev_i, non_blocking=True)
        torch.cuda.current_stream(env.device).synchronize()
        hf, hi = self._host_f.numpy(), self._host_i.numpy()
        F = self.spec.num_features
        o = hf[:N * F].reshape(N, F).copy()
        r = hf[N * F:N * F + self._nr].copy()
        profit = hf[N * F + self._nr:].copy()
        order, dem, acq, ship = (hi[j * N:(j + 1) * N] for j in range(4))
        inv, bl, ou = (hi[(6 + j) * N:(7 + j) * N] for j in range(3))
        if not self.serial and hi[9 * N]:
            raise Exception("Infinite Loop (divergent shipment split guard, IM_div_env.py:424-498)")
        self.order_r[t] = order
        self.demand[t] = dem
        self.ship[t] = ship
        self.acquisition[t] = acq
        self.inv[t + 1] = inv
        self.backlog[t + 1] = bl
        self.order_u[t + 1] = ou
        return self._finish(t, o, r, profit)

    def close(self):
        self._env.close()


class _SingleAgent(_Adaptor, _GymEnv):
    def _wrap_obs(self, o):
        return o.copy()

    def _actions(self, action):
        a = np.squeeze(np.asarray(action, dtype=np.float64))
        return np.broadcast_to(a, (self.num_nodes,)).astype(np.float64)

    def _finish(self, t, o, r, profit):
        info = {"period": t, "demand": self.demand[t, :], "ship": self.ship[t, :],
                "acquisition": self.acquisition[t, :], "profit": profit}
        self.period += 1
        self.state = o.copy()
        done = self.period >= self.num_periods
        return self.state, np.float64(r[0]), done, info


class _MultiAgent(_Adaptor, _MultiAgentEnv):
    PREFIX = None

    def __init__(self, config, device=None):
        build = build_spec(self.KIND, config)
        n = build.num_nodes
        self.agent_names = [self.PREFIX + str(i) for i in range(n)]
        self.num_agents = int(config.get("num_agents", n))
        _Adaptor.__init__(self, config, device)

    def _wrap_obs(self, o):
        return {name: o[i].copy() for i, name in enumerate(self.agent_names)}

    def _actions(self, action_dict):
        return np.array([float(np.asarray(action_dict[name], dtype=np.float64).reshape(-1)[0])
                         for name in self.agent_names])

    def _finish(self, t, o, r, profit):
        self.period += 1
        self.state = self._wrap_obs(o)
        if self.spec.reward_mode == nat.REWARD_INDEPENDENT:
            rewards = {name: np.float64(r[i]) for i, name in enumerate(self.agent_names)}
        else:
            rewards = {name: np.float64(r[0]) for name in self.agent_names}
        done = {"__all__": self.period >= self.num_periods}
        info = {}
        for i, name in enumerate(self.agent_names):
            info[name] = {"period": self.period, "demand": self.demand[t, i], "ship": self.ship[t, i],
                          "acquisition": self.acquisition[t, i], "actual order": self.order_r[t, i],
                          "profit": profit[i]}
        return self.state, rewards, done, info


class InvManagement(_SingleAgent):
    """environments/IM_env.py:InvManagement (serial supply chain, single agent)."""
    KIND = "IM"


class InvManagementDiv(_SingleAgent):
    """environments/IM_div_env.py:InvManagementDiv (divergent network, single agent)."""
    KIND = "IM_div"


class MultiAgentInvManagement(_MultiAgent):
    """environments/MAIM_env.py:MultiAgentInvManagement (serial, one agent per stage)."""
    KIND = "MAIM"
    PREFIX = "stage_"

    @property
    def stage_names(self):
        return self.agent_names


class MultiAgentInvManagementDiv(_MultiAgent):
    """environments/MAIM_div_env.py:MultiAgentInvManagementDiv (divergent, one agent per node)."""
    KIND = "MAIM_div"
    PREFIX = "node_"

    @property
    def node_names(self):
        return self.agent_names


__all__ = ["InvManagement", "MultiAgentInvManagement", "InvManagementDiv", "MultiAgentInvManagementDiv",
           "rescale", "rev_scale", "make_spaces"]

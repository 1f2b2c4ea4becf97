"""Base-stock (order-up-to) policy evaluation on the GPU.

Replaces, batched, the reference's policy-search loop in base_restock_policy.py:

  base_stock_policy(policy, env)        :4-21   order up to `policy` at every node
  dfo_func(policy, env, demand=None)    :24-45  one episode -> -1/T * sum(pmf(demand) * rewards)
  optimize_inventory_policy(env, fun, init_policy=None, method='Powell', demand=None)  :48-63

and the base-stock evaluation loop of the experiment scripts (inv_management.py:222-232,
inv_management_div.py). ``BaseStockRollout`` runs P policies x S demand scenarios as P*S whole
episodes in ONE fused kernel launch (imenv_base_stock_rollout: state in registers, lead-time queue
in LDS, wavefront reductions of the metrics), so a population / grid of candidate policies is
scored in one call instead of P*S Python episodes.

The module-level functions keep the reference's names, arguments and results so that a script
importing them from here instead of base_restock_policy runs unchanged on the drop-in env
adaptors (envs.py): ``dfo_func`` returns the same float64 objective bit for bit (the GPU computes
the reference's expression in its operation order, np.sum's pairwise order included), so Powell
takes the same path and ``optimize_inventory_policy`` returns the same policy.
"""
from ctypes import byref, c_void_p

import numpy as np
import torch
from scipy.optimize import minimize
from scipy.stats import poisson, randint

from . import _native as nat
from .spec import HostSpec


def demand_pmf(spec, max_value):
    """pmf table [0, max_value] of the spec's demand distribution: env.dist.pmf(k, **env.dist_param)
    (base_restock_policy.py:42), evaluated by the reference's own SciPy distribution per value."""
    k = np.arange(int(max_value) + 1)
    if spec.demand_dist == "poisson":
        return poisson.pmf(k, mu=spec.mu).astype(np.float64)
    if spec.demand_dist == "uniform":
        low, high = spec.lower_upper[:2]
        return randint.pmf(k, low=low, high=high).astype(np.float64)
    return None     # "custom": the reference env has no `dist` (dfo_func raises AttributeError)


class BaseStockRollout:
    """Batched base-stock episodes of one env spec on one GPU.

        ro = BaseStockRollout("IM", dfo_config)
        out = ro.run(policies, demand=test_demand)        # policies [P, N], demand [S, T] / [S, R, T]
        out["objective"]       # [P, S] dfo_func values
        out["return"]          # [P, S] episode rewards (the evaluation loop's dfo_rewards)
        out["stats"]           # [P, 5, 2]: np.mean / np.std over the S scenarios per metric

    Demand is the reference's reset(customer_demand=...) table per scenario, or None to draw it
    in-kernel (Philox keyed by (spec seed, scenario_offset + s, episode), the same draws
    VectorInvEnv.reset() makes for env id s).
    """

    def __init__(self, kind_or_spec, config=None, device=None):
        # the handle supplies spec, device and kernel cache; its own env state is unused (1 env)
        from .vector_env import VectorInvEnv
        self._env = VectorInvEnv(kind_or_spec, config, n_envs=1, device=device)
        self.spec = self._env.spec
        self.device = self._env.device
        self.N, self.R, self.T = self._env.N, self._env.R, self._env.T
        self._pmf = None
        self._pmf_max = -1

    def _pmf_table(self, max_value):
        if max_value > self._pmf_max:
            tab = demand_pmf(self.spec, max_value)
            if tab is None:
                return None
            self._pmf = torch.as_tensor(tab, device=self.device)
            self._pmf_max = int(max_value)
        return self._pmf

    def _demand_table(self, demand):
        """[S, T] (serial) / [S, R, T] (tree) or [T] / [R, T] for one scenario -> device int32 [T][R][S]."""
        d = torch.as_tensor(np.asarray(demand) if not torch.is_tensor(demand) else demand)
        R, T = self.R, self.T
        if d.dim() == 1 or (d.dim() == 2 and not self.spec.serial and d.shape == (R, T)):
            d = d.unsqueeze(0)
        if d.dim() == 2:
            d = d.unsqueeze(1)
        if d.dim() != 3 or d.shape[1] != R or d.shape[2] < T:
            raise ValueError("demand must be [S, T] (serial) or [S, R, T] (tree), got %s" % (tuple(d.shape),))
        return d[:, :, :T].to(device=self.device, dtype=torch.int32).permute(2, 1, 0).contiguous()

    def run(self, policies, demand=None, n_scenarios=None, scenario_offset=0, episode=0, noisy_delay=False,
            noisy_delay_threshold=0.0, objective=True, per_episode=True, stream=None, check_finite=True):
        """check_finite: raise ValueError for non-finite policies. Host inputs are checked on the host;
        a device tensor costs a device-to-host sync per call (a caller that validated its tensor once,
        e.g. a timing loop, passes False)."""
        if check_finite and not torch.is_tensor(policies) and not np.isfinite(np.asarray(policies, dtype=np.float64)).all():
            raise ValueError("policies must be finite")
        p = torch.as_tensor(policies, dtype=torch.float64, device=self.device)
        if p.dim() == 1:
            p = p.unsqueeze(0)
        if p.dim() != 2 or p.shape[1] != self.N:
            raise ValueError("policies must be [P, %d]" % self.N)
        if check_finite and torch.is_tensor(policies) and not torch.isfinite(p).all():
            raise ValueError("policies must be finite")
        p = p.contiguous()
        P = p.shape[0]
        table = None
        if demand is not None:
            table = self._demand_table(demand)
            S = table.shape[2]
            dmax = int(table.max().item()) if table.numel() else 0
        else:
            if n_scenarios is None:
                raise ValueError("n_scenarios is required when demand is drawn in-kernel")
            S = int(n_scenarios)
            if self.spec.demand_dist == "poisson":
                dmax = int(len(self._env.poisson_table()))
            else:
                dmax = int(self.spec.lower_upper[1])
            if self.spec.noisy_demand:
                dmax *= 2
        pmf = self._pmf_table(max(dmax, 0)) if objective else None
        ep = torch.empty((nat.NUM_STATS, P, S), dtype=torch.float64, device=self.device) if per_episode else None
        stats = torch.empty((P, nat.NUM_STATS, 2), dtype=torch.float64, device=self.device)
        a = nat.ImEnvRollout()
        a.policy = p.data_ptr()
        a.num_policies = P
        a.num_scenarios = S
        a.demand = table.data_ptr() if table is not None else None
        a.scenario_offset = int(scenario_offset)
        a.episode = int(episode)
        a.demand_pmf = pmf.data_ptr() if pmf is not None else None
        a.pmf_len = int(pmf.numel()) if pmf is not None else 0
        a.noisy_delay = 1 if noisy_delay else 0
        a.noisy_delay_threshold = float(noisy_delay_threshold)
        a.episode_stats = ep.data_ptr() if ep is not None else None
        a.policy_stats = stats.data_ptr()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        nat.check(self._env.lib.imenv_base_stock_rollout(self._env._h, byref(a), c_void_p(st.cuda_stream)),
                  "imenv_base_stock_rollout")
        # keep inputs alive until the stream has consumed them (torch's caching allocator is stream-aware
        # for the current stream; record_stream covers a caller-supplied one)
        for t in (p, table, pmf):
            if t is not None:
                t.record_stream(st)
        out = {"stats": stats}
        if ep is not None:
            for k, name in enumerate(nat.STAT_NAMES):
                out[name] = ep[k]
        return out

    def kernel_info(self):
        return self._env.kernel_info()

    def close(self):
        self._env.close()


# ---------------------------------------------------------------- drop-in functions
def base_stock_policy(policy, env):
    """base_restock_policy.py:4-21 on an env exposing inv / order_u / backlog histories, order_max
    and num_nodes (the drop-in adaptors of envs.py do): order up to `policy` at every node."""
    t = env.period
    inv_ech = env.inv[t, :] + env.order_u[t, :] - env.backlog[t, :]
    return np.minimum(env.order_max, np.maximum(policy - inv_ech, np.zeros(env.num_nodes)))


def _rollout_for(env):
    ro = getattr(env, "_base_stock_rollout", None)
    if ro is None:
        spec = getattr(env, "spec", None)
        if not isinstance(spec, HostSpec):
            raise TypeError("dfo_func needs an imenv env (envs.py adaptor or a HostSpec holder)")
        dev = getattr(getattr(env, "_env", None), "device", None)
        ro = BaseStockRollout(spec, device=dev)
        env._base_stock_rollout = ro
    return ro


def dfo_func(policy, env, demand=None, *args):
    """base_restock_policy.py:24-45 on the GPU: one episode of the base-stock policy from a fresh
    reset, returning -1/T * np.sum(pmf(customer_demand) * rewards). With demand=None the episode's
    demand is drawn the way env.reset() draws it (the adaptor's host RNG stream, as the reference)."""
    ro = _rollout_for(env)
    if demand is None:
        demand = env._draw_demand()
    out = ro.run(np.asarray(policy, dtype=np.float64)[None, :], demand=np.asarray(demand)[None], objective=True,
                 per_episode=True)
    return float(out["objective"][0, 0].item())


def optimize_inventory_policy(env, fun=dfo_func, init_policy=None, method="Powell", demand=None):
    """base_restock_policy.py:48-63: scipy.optimize.minimize of `fun` from init_policy (default
    mu at every stage), then the policy rounded to non-negative integers."""
    if init_policy is None:
        init_policy = np.ones(env.num_stages) * env.mu
    if demand is None:
        out = minimize(fun=fun, x0=init_policy, args=env, method=method)
    else:
        out = minimize(fun=fun, x0=init_policy, args=(env, demand), method=method)
    policy = out.x.copy()
    policy = np.round(np.maximum(policy, 0), 0).astype(int)
    return policy, out


def evaluate_base_stock(env, policy, test_demand, noisy_delay=False, noisy_delay_threshold=0.0):
    """The base-stock evaluation loop (inv_management.py:222-232): one episode per test-demand row,
    returning the list of episode rewards (dfo_rewards) — all rows in one launch."""
    ro = _rollout_for(env)
    out = ro.run(np.asarray(policy, dtype=np.float64)[None, :], demand=test_demand, objective=False,
                 noisy_delay=noisy_delay, noisy_delay_threshold=noisy_delay_threshold)
    return out["return"][0].cpu().numpy()

"""Open-loop plan replay on the GPU: the LP scripts' evaluation loop, batched.

Every LP / planning script of the reference (SHLP_8.py:737-766; the same loop in SHLP.py, SHLP_2.py,
SHLP_div1.py:570-597, SHLP_div2.py, DSHLP*.py, Oracle*.py, DecLP.py, Distributed*_LP.py) scores its
plans by replaying them through the env, one scenario at a time:

    s = LP_env.reset(customer_demand=LP_demand[j])
    while not done:
        s, r, done, info = LP_env.step(SHLP_actions[t, :])
        profit[j, t] = r
        total_inventory += sum(s[:, 0]); total_backlog += sum(s[:, 1]); customer_backlog += s[0, 1]
        lp_reward += r

``PlanRollout`` runs P plans x S scenarios of that loop as P*S whole episodes in ONE fused kernel
launch (imenv_plan_rollout: the rollout kernel with the plan as its action source, state in
registers, the lead-time queue in LDS). Two plan layouts:

  shared       plans [P, T, N]: plan p is replayed on every scenario (a fixed plan's robustness)
  per-episode  plans [S, T, N] or [P, S, T, N]: scenario j replays its own plan, as the scripts
               do when they solve the LP per demand scenario (SHLP_actions of scenario j)

``replay_plans`` keeps the scripts' result names (lp_reward_list, inventory_list, backlog_list,
customer_backlog_list, profit).
"""
from ctypes import byref, c_void_p

import numpy as np
import torch

from . import _native as nat


class PlanRollout:
    """Batched plan replays of one env spec on one GPU.

        pr = PlanRollout("IM", lp_config)
        out = pr.run(plans, demand=LP_demand, per_episode=True)   # plans [S, T, N], demand [S, T]
        out["return"]      # [P, S] lp_reward per episode
        out["rewards"]     # [P, S, T] profit[j, t]
        out["stats"]       # [P, 5, 2] np.mean / np.std over the S scenarios per metric
    """

    def __init__(self, kind_or_spec, config=None, device=None):
        # the handle supplies spec, device and kernel cache; its own env state is unused (1 env)
        from .policy import BaseStockRollout
        self._ro = BaseStockRollout(kind_or_spec, config, device=device)
        self._env = self._ro._env
        self.spec, self.device = self._ro.spec, self._ro.device
        self.N, self.R, self.T = self._ro.N, self._ro.R, self._ro.T

    def _plans(self, plans, per_episode, S):
        """-> (device tensor in the kernel's layout, P): shared [P][T][N]; per-episode [T][P][S][N]."""
        x = plans if torch.is_tensor(plans) else torch.as_tensor(np.asarray(plans))
        if x.dtype not in (torch.float32, torch.float64):
            x = x.to(torch.float64)
        N, T = self.N, self.T
        if per_episode:
            if x.dim() == 3:
                x = x.unsqueeze(0)
            if x.dim() != 4 or x.shape[2] < T or x.shape[3] != N or (S is not None and x.shape[1] != S):
                raise ValueError("per-episode plans must be [S, T, %d] or [P, S, T, %d], got %s"
                                 % (N, N, tuple(x.shape)))
            x = x[:, :, :T].to(self.device).permute(2, 0, 1, 3).contiguous()
            return x, x.shape[1], x.shape[2]
        if x.dim() == 2:
            x = x.unsqueeze(0)
        if x.dim() != 3 or x.shape[1] < T or x.shape[2] != N:
            raise ValueError("shared plans must be [T, %d] or [P, T, %d], got %s" % (N, N, tuple(x.shape)))
        x = x[:, :T].to(self.device).contiguous()
        return x, x.shape[0], S

    def run(self, plans, demand=None, per_episode=False, n_scenarios=None, scenario_offset=0, episode=0,
            noisy_delay=False, noisy_delay_threshold=0.0, rewards=True, per_episode_stats=True, stream=None):
        table = self._ro._demand_table(demand) if demand is not None else None
        S = table.shape[2] if table is not None else (None if n_scenarios is None else int(n_scenarios))
        x, P, S2 = self._plans(plans, per_episode, S)
        S = S if S is not None else S2
        if S is None:
            raise ValueError("n_scenarios is required for shared plans when demand is drawn in-kernel")
        if table is None and self.spec.demand_dist not in ("poisson", "uniform"):
            raise ValueError("custom demand needs a demand table")
        rew = torch.empty((self.T, P, S), dtype=torch.float64, device=self.device) if rewards else None
        ep = torch.empty((nat.NUM_STATS, P, S), dtype=torch.float64, device=self.device) if per_episode_stats else None
        stats = torch.empty((P, nat.NUM_STATS, 2), dtype=torch.float64, device=self.device)
        a = nat.ImEnvPlanRollout()
        a.actions = x.data_ptr()
        a.action_dtype = nat.F64 if x.dtype == torch.float64 else nat.F32
        a.plan_layout = nat.PLAN_PER_EPISODE if per_episode else nat.PLAN_SHARED
        a.num_plans = P
        a.num_scenarios = S
        a.demand = table.data_ptr() if table is not None else None
        a.scenario_offset = int(scenario_offset)
        a.episode = int(episode)
        a.noisy_delay = 1 if noisy_delay else 0
        a.noisy_delay_threshold = float(noisy_delay_threshold)
        a.rewards = rew.data_ptr() if rew is not None else None
        a.episode_stats = ep.data_ptr() if ep is not None else None
        a.policy_stats = stats.data_ptr()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        nat.check(self._env.lib.imenv_plan_rollout(self._env._h, byref(a), c_void_p(st.cuda_stream)),
                  "imenv_plan_rollout")
        for t in (x, table):
            if t is not None:
                t.record_stream(st)
        out = {"stats": stats}
        if rew is not None:
            out["rewards"] = rew.permute(1, 2, 0)      # [P, S, T] view of the [T][P][S] rows
        if ep is not None:
            for k, name in enumerate(nat.STAT_NAMES):
                if name != "objective":
                    out[name] = ep[k]
        return out

    def kernel_info(self):
        return self._env.kernel_info()

    def close(self):
        self._ro.close()


def replay_plans(env_or_spec, plans, demand, per_episode=True, config=None, device=None):
    """The LP scripts' replay loop (SHLP_8.py:737-766) for every scenario at once. plans: per-episode
    [S, T, N] (scenario j's SHLP_actions) or shared [T, N]; demand: LP_demand [S, T] / [S, R, T].
    Returns the scripts' lists (lp_reward_list, inventory_list, backlog_list, customer_backlog_list)
    as NumPy arrays and profit [S, T]."""
    spec = getattr(env_or_spec, "spec", env_or_spec)
    # a drop-in adaptor holds its VectorInvEnv in ._env; a VectorInvEnv has .device itself
    dev = device if device is not None else getattr(getattr(env_or_spec, "_env", env_or_spec), "device", None)
    pr = PlanRollout(spec, config, device=dev)
    try:
        out = pr.run(plans, demand=demand, per_episode=per_episode)
        return dict(lp_reward_list=out["return"][0].cpu().numpy(),
                    inventory_list=out["inventory"][0].cpu().numpy(),
                    backlog_list=out["backlog"][0].cpu().numpy(),
                    customer_backlog_list=out["customer_backlog"][0].cpu().numpy(),
                    profit=out["rewards"][0].cpu().numpy())
    finally:
        pr.close()

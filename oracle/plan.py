"""Open-loop plan replays on the CPU restatement. TEST INFRASTRUCTURE ONLY.

Restates the LP scripts' evaluation loop over OracleEnv, the checker for imenv_plan_rollout /
imenv.plan. SHLP_8.py:737-766 (the same loop is in SHLP*.py, DSHLP*.py, Oracle*.py, DecLP.py,
Distributed*_LP.py):

    s = LP_env.reset(customer_demand=LP_demand[j])
    while not done:
        s, r, done, info = LP_env.step(SHLP_actions[t, :])
        profit[j, t] = r
        total_inventory += sum(s[:, 0]); total_backlog += sum(s[:, 1]); customer_backlog += s[0, 1]
        lp_reward += r

The scripts run with standardise_state False, so s[:, 0] / s[:, 1] are the integer inventory and
backlog after the step; the restatement sums the state (exact integers, as the scripts' float64
sums of integers are). Pinned by tests/golden/plan_replay.npz (tools/gen_plan_fixtures.py runs that
loop on the reference's own env classes).
"""
import numpy as np

from .base_stock import STAT_NAMES
from .im_oracle import OracleEnv


def plan_rollout(kind, config, plans, per_episode=False, demand=None, n_scenarios=None, rng=None,
                 noisy_delay=False, noisy_delay_threshold=0.0):
    """plans: [P, T, N] (one plan per row, replayed on every scenario) or, with per_episode,
    [T, P, S, N] (each episode its own plan). demand [S, T] / [S, R, T] or None with rng (Philox
    draws keyed like the product's). Returns {name: [P, S]} for STAT_NAMES (objective 0) plus
    "rewards" [T, P, S]."""
    plans = np.asarray(plans, dtype=np.float64)
    P = plans.shape[1] if per_episode else plans.shape[0]
    S = int(np.asarray(demand).shape[0]) if demand is not None else int(n_scenarios)
    out = {k: np.zeros((P, S)) for k in STAT_NAMES}
    rewards = None
    for p in range(P):
        env = OracleEnv(kind, config, n_envs=S)
        env.reset(customer_demand=demand, rng=rng, noisy_delay=noisy_delay,
                  noisy_delay_threshold=noisy_delay_threshold)
        T = env.num_periods
        if rewards is None:
            rewards = np.zeros((T, P, S))
        ret = np.zeros(S)
        for t in range(T):
            act = plans[t, p] if per_episode else np.broadcast_to(plans[p, t], (S, env.N))
            _, r, _, _ = env.step(np.array(act))
            r = np.asarray(r, dtype=np.float64).reshape(S)
            rewards[t, p] = r                          # profit[j, t] = r
            ret = ret + r                              # lp_reward += r
            nxt = env.state_arrays()
            out["inventory"][p] += nxt["inv"].sum(axis=1)          # sum(s[:, 0])
            out["backlog"][p] += nxt["backlog"].sum(axis=1)        # sum(s[:, 1])
            out["customer_backlog"][p] += nxt["backlog"][:, 0]     # s[0, 1]
        out["return"][p] = ret
    out["rewards"] = rewards
    return out

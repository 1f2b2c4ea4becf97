"""The reference's evaluation-harness accumulation. TEST INFRASTRUCTURE ONLY.

Restates the per-episode sums of the test loops in inv_management.py:567-606 (single agent) and
MA_inv_management.py:517-587 / MA_inv_management_div.py:520-560 (multi agent), evaluated on an
episode's float64 observations, rewards and info["profit"]; the checker for
imenv_set_episode_metrics (the step kernel's harness accumulators) and imenv_column_stats.
"""
import numpy as np


def rev_scale(val_scaled, min_val, max_val, A=-1, B=1):
    """IM_env.py:446-456."""
    return ((val_scaled - A) * (max_val - min_val)) / (B - A) + min_val


def harness_metrics(obs, reward, profit, inv_max, a, b, multi_agent):
    """obs [E, T, N, F] float64 (after each step), reward [E, T, 1] (single agent) or [E, T, N]
    (each agent's), profit [E, T, N]. Returns [E, 4 + N]: episode reward, total inventory, total
    backlog, customer backlog, stage rewards — in the harness's own accumulation order."""
    E, T, N = profit.shape
    out = np.zeros((E, 4 + N))
    for e in range(E):
        episode_reward = 0
        total_inventory = 0
        total_backlog = 0
        customer_backlog = 0
        stage = np.zeros(N)
        for t in range(T):
            o = obs[e, t]
            if multi_agent:                         # MA_inv_management.py:559-572
                total_step_inv = 0
                total_step_bl = 0
                for m in range(N):
                    episode_reward += reward[e, t, m]
                    stage[m] += profit[e, t, m]
                    total_step_inv += rev_scale(o[m][0], 0, inv_max[m], a, b)
                    total_step_bl += rev_scale(o[m][1], 0, inv_max[m], a, b)
                total_inventory += total_step_inv
                total_backlog += total_step_bl
                customer_backlog += rev_scale(o[0][1], 0, inv_max[0], a, b)
            else:                                   # inv_management.py:586-597
                inv = rev_scale(o[:, 0], np.zeros(N), inv_max, a, b)
                bl = rev_scale(o[:, 1], np.zeros(N), inv_max, a, b)
                total_inventory += sum(inv)
                total_backlog += sum(bl)
                customer_backlog += bl[0]
                for m in range(N):
                    stage[m] += profit[e, t, m]
                episode_reward += reward[e, t, 0]
        out[e, 0] = episode_reward
        out[e, 1] = total_inventory
        out[e, 2] = total_backlog
        out[e, 3] = customer_backlog
        out[e, 4:] = stage
    return out

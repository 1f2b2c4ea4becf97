"""Centralised-critic observation restatement. TEST INFRASTRUCTURE ONLY.

central_critic_observer (models/CC_Model.py:196-214) per agent dict {own_obs, opponent_obs (others'
obs concatenated in agent order), opponent_action}, with the opponent actions FillInActions
(:165-193) writes (np.clip(a, -1, 1), or [a, b] in CC_inv_management.py:403), flattened in RLlib's
sorted-key Dict order. Pinned by tests/golden/cc_obs.npz (the reference function's own output,
tools/gen_cc_fixtures.py).
"""
import numpy as np


def cc_observation(obs, actions=None, lo=-1.0, hi=1.0):
    """obs [B, N, F], actions [B, N] or None -> [B, N, N*F + N - 1]."""
    obs = np.asarray(obs)
    B, N, F = obs.shape
    out = np.zeros((B, N, N * F + N - 1), dtype=obs.dtype)
    for m in range(N):
        others = [o for o in range(N) if o != m]
        if actions is not None:
            out[:, m, :N - 1] = np.clip(np.asarray(actions)[:, others], lo, hi)
        out[:, m, N - 1:(N - 1) * (F + 1)] = obs[:, others, :].reshape(B, -1)
        out[:, m, (N - 1) * (F + 1):] = obs[:, m, :]
    return out

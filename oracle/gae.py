"""GAE restatement. TEST INFRASTRUCTURE ONLY.

RLlib 1.5's compute_advantages (use_gae=True) and discount_cumsum, as the trainers' postprocessing
calls them (models/CC_Policy.py:238-250, gamma / lambda of utils.py:19-23). RLlib is not installed
here: this follows its published algorithm (ray/rllib/evaluation/postprocessing.py) with the same
NumPy / SciPy calls, for one trajectory per env. Parity vs RLlib itself is unpinned (no RLlib
fixtures exist); the checker for imenv_gae.
"""
import numpy as np
import scipy.signal


def discount_cumsum(x, gamma):
    return scipy.signal.lfilter([1], [1, float(-gamma)], x[::-1], axis=0)[::-1]


def compute_advantages(rewards, vf_preds, last_r, gamma, lambda_):
    """One trajectory: rewards [T], vf_preds [T] -> (advantages f32 [T], value_targets f32 [T])."""
    vpred_t = np.concatenate([vf_preds, np.array([last_r])])
    delta_t = rewards + gamma * vpred_t[1:] - vpred_t[:-1]
    adv = discount_cumsum(delta_t, gamma * lambda_)
    value_targets = (adv + vf_preds).astype(np.float32)
    return adv.astype(np.float32), value_targets


def gae_batch(rewards, values, last_value=None, gamma=0.99, lambda_=0.95):
    """[T, n] buffers (one completed trajectory per env when last_value is None)."""
    T, n = rewards.shape
    adv = np.zeros((T, n), dtype=np.float32)
    vt = np.zeros((T, n), dtype=np.float32)
    for e in range(n):
        last_r = 0.0 if last_value is None else last_value[e]
        adv[:, e], vt[:, e] = compute_advantages(rewards[:, e], values[:, e], last_r, gamma, lambda_)
    return adv, vt

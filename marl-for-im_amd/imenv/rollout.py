"""GPU-resident rollout buffer and GAE for the trainers around the env.

RLlib's sampler collects env steps into numpy SampleBatches on the host and postprocesses each
trajectory with compute_advantages (models/CC_Policy.py:238-250). Here the whole [T, n] rollout
stays in HBM: the env writes observations and rewards straight into the buffer
(VectorInvEnv.step(obs_out=..., reward_out=...)), the policy writes actions and values, and
``gae`` (imenv_gae) computes advantages and value targets for every env in one launch.
"""
import torch

from . import _native as nat


def gae(rewards, values, last_value=None, gamma=0.99, lambda_=0.95, value_targets=True):
    """rewards, values: [T, n] device tensors (float32/float64); last_value: [n] bootstrap values or
    None for completed episodes. Returns (advantages, value_targets) float32 [T, n]."""
    if rewards.shape != values.shape or rewards.dim() != 2:
        raise ValueError("rewards and values must both be [T, n]")
    T, n = rewards.shape
    r = rewards.contiguous()
    v = values.contiguous()
    lv = None
    if last_value is not None:
        lv = last_value.to(dtype=v.dtype, device=v.device).contiguous()
        if lv.shape != (n,):
            raise ValueError("last_value must be [n]")
    code = {torch.float32: nat.F32, torch.float64: nat.F64}
    if r.dtype not in code or v.dtype not in code:
        raise ValueError("float32 / float64 only")
    adv = torch.empty((T, n), dtype=torch.float32, device=r.device)
    vt = torch.empty((T, n), dtype=torch.float32, device=r.device) if value_targets else None
    st = torch.cuda.current_stream(r.device).cuda_stream
    nat.check(nat.load().imenv_gae(n, T, r.data_ptr(), code[r.dtype], v.data_ptr(), code[v.dtype],
                                   lv.data_ptr() if lv is not None else None, float(gamma), float(lambda_),
                                   adv.data_ptr(), vt.data_ptr() if vt is not None else None, st), "imenv_gae")
    return adv, vt


class RolloutBuffer:
    """[T, n] episode storage on the env's device, shaped for VectorInvEnv.step's output arguments.

        buf = RolloutBuffer(env)                    # T = env.T periods, n = env.n envs
        env.reset(obs_out=buf.obs[0])
        for t in range(env.T):
            a, v = policy(buf.obs[t])
            buf.actions[t], buf.values[t] = a, v
            buf.step(t)                             # = env.step(buf.actions[t], obs_out=buf.obs[t + 1], ...)
        adv, vt = buf.advantages()

    buf.step(t) launches period t through the env's rollout_stepper (buffers checked once, one C call).
    obs / actions / rewards are fixed for the buffer's life (the stepper holds their pointers): write
    into them (buf.actions[t] = a), never rebind them (read-only properties).
    """

    def __init__(self, env, obs_dtype=torch.float32):
        # rewards are float64, the dtype the env writes (the reference's profit arithmetic)
        T, n, N, F = env.T, env.n, env.N, env.F
        dev = env.device
        self._obs = torch.empty((T + 1, n, N, F), dtype=obs_dtype, device=dev)
        self._actions = torch.empty((T, n, N), dtype=torch.float32, device=dev)
        self._rewards = torch.empty((T,) + tuple(env.reward_shape()), dtype=torch.float64, device=dev)
        self.values = torch.empty((T, n), dtype=torch.float32, device=dev)
        self._stepper = env.rollout_stepper(self._actions, self._obs, self._rewards)

    obs = property(lambda self: self._obs, doc="[T + 1, n, N, F] observations (row 0: reset)")
    actions = property(lambda self: self._actions, doc="[T, n, N] float32 actions")
    rewards = property(lambda self: self._rewards, doc="[T] + reward_shape float64 rewards")

    def step(self, t):
        """Step period t of the bound env from actions[t] into obs[t + 1] and rewards[t]; returns done."""
        return self._stepper(t)

    def advantages(self, gamma=0.99, lambda_=0.95, last_value=None):
        r = self.rewards if self.rewards.dim() == 2 else self.rewards.sum(-1)
        return gae(r, self.values, last_value, gamma, lambda_)

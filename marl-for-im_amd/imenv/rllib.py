"""Batched RLlib surfaces: n envs of one RLlib rollout worker stepped by ONE kernel launch per step.

The reference trains with RLlib 1.5 (poetry.lock), registering one env object per creator call
(inv_management.py:72-78, MA_inv_management.py:83-84); a worker with num_envs_per_worker = n then
holds n such objects and steps them one by one in Python. These classes are that batch as one object
over one VectorInvEnv, with the call shapes RLlib's sampler uses:

- ``InvVectorEnv`` — ray.rllib.env.VectorEnv for the single-agent classes (InvManagement,
  InvManagementDiv): ``num_envs``, ``observation_space`` / ``action_space`` (one env's),
  ``vector_reset()``, ``reset_at(i)``, ``vector_step(actions)``, ``get_unwrapped()``. RLlib wraps a
  VectorEnv in its own BaseEnv adapter.
- ``InvMultiAgentBaseEnv`` — ray.rllib.env.BaseEnv for the multi-agent classes
  (MultiAgentInvManagement, MultiAgentInvManagementDiv): ``poll()``, ``send_actions(action_dict)``,
  ``try_reset(env_id)``, ``get_unwrapped()``, ``stop()``, with {env_id: {agent_id: value}} dicts and
  "__all__", released exactly as RLlib's _MultiAgentEnvToBaseEnv releases them for n separate
  MultiAgentEnv objects (initial rewards None, infos {}; rewards / dones / infos of an agent only with
  its observation).

Per step: the actions of all n envs go to the device in one copy, one step-kernel launch advances
every env, and observations, rewards and the info fields come back in one copy. Values are the
reference's (float64 observations, the info keys period / demand / ship / acquisition / profit and,
multi-agent, 'actual order'), checked bit for bit against the reference's golden sessions
(tests/test_rllib_gpu.py).

Lockstep: every env of the batch shares the period (the reference's envs all have the same fixed
horizon and no auto-reset), so all n episodes end together. RLlib then resets the envs one by one
(reset_at / try_reset); the first such call runs one batched reset and the others return their env's
row of it. Resetting an env in the middle of the batch's episode is refused (RuntimeError).

Randomness: by default demand is drawn in-kernel (Philox keyed by the spec's seed, the global env id
and the episode), so the n envs of a worker and the workers of a job (``env_offset``, e.g.
worker_index * n) draw independent streams. ``episode_inputs(episode) -> dict`` can instead supply the
reset's customer_demand / noisy_delay / noisy_delay_threshold / delay_uniforms (VectorInvEnv.reset
keywords), e.g. the reference's own demand tables.
"""
import numpy as np
import torch

from . import _native as nat
from .envs import make_spaces
from .spec import build_spec
from .vector_env import VectorInvEnv

try:  # pragma: no cover - base classes only where RLlib is installed
    from ray.rllib.env.vector_env import VectorEnv as _VectorEnv
except Exception:
    _VectorEnv = object
try:  # pragma: no cover
    from ray.rllib.env.base_env import BaseEnv as _BaseEnv
except Exception:
    _BaseEnv = object


class _Batch:
    """One VectorInvEnv of n envs with pinned host mirrors of everything a step returns."""

    def __init__(self, kind, config, num_envs, device=None, env_offset=0, info=True, episode_inputs=None):
        self.spec = build_spec(kind, dict(config))
        if env_offset is None:
            env_offset = int(getattr(config, "worker_index", 0)) * int(num_envs)   # RLlib EnvContext
        self.env = VectorInvEnv(self.spec, n_envs=num_envs, device=device, env_offset=env_offset,
                                obs_dtype=torch.float64)
        self.n, self.N, self.F, self.T = self.env.n, self.env.N, self.env.F, self.env.T
        self.info = bool(info)
        self.episode_inputs = episode_inputs
        self.observation_space, self.action_space = make_spaces(kind, self.spec)
        n, N, F = self.n, self.N, self.F
        dev = self.env.device
        self.nr = N if self.spec.reward_mode == nat.REWARD_INDEPENDENT else 1
        # one float64 and one int32 device buffer, each copied to pinned host memory once per step
        self._dev_f = torch.empty(n * N * F + n * self.nr + n * N, dtype=torch.float64, device=dev)
        self._dev_i = torch.empty(6 * n * N, dtype=torch.int32, device=dev)
        pin = dev.type == "cuda"     # (the CPU tests drive this class over an oracle-backed stand-in)
        self._host_f = torch.empty(self._dev_f.shape, dtype=torch.float64, pin_memory=pin)
        self._host_i = torch.empty(self._dev_i.shape, dtype=torch.int32, pin_memory=pin)
        self._host_a = torch.empty((n, N), dtype=torch.float64, pin_memory=pin)
        self._dev_a = torch.empty((n, N), dtype=torch.float64, device=dev)
        f, i = self._dev_f, self._dev_i
        self._obs = f[:n * N * F].view(n, N, F)
        self._rew = f[n * N * F:n * N * F + n * self.nr].view((n, N) if self.nr == N else (n,))
        iv = lambda j: i[j * n * N:(j + 1) * n * N].view(n, N)
        self._info = dict(order=iv(0), demand=iv(1), acquisition=iv(2), ship=iv(3),
                          profit=f[n * N * F + n * self.nr:].view(n, N), ship_to=iv(4), backlog_to=iv(5))
        self.episode = -1
        self.done = False          # the batch's episode has ended (all envs at period T)
        self.reset_obs = None      # host [n, N, F] of the last batched reset
        self.reset_taken = None    # which envs have been handed their row of it

    def _sync_copy(self, what):
        self._host_f.copy_(self._dev_f, non_blocking=True)
        if what:
            self._host_i.copy_(self._dev_i, non_blocking=True)
        if self.env.device.type == "cuda":
            torch.cuda.current_stream(self.env.device).synchronize()

    def reset_all(self):
        """One batched reset: every env to period 0; returns host observations [n, N, F] (float64)."""
        kw = self.episode_inputs(self.episode + 1) if self.episode_inputs is not None else {}
        self.env.reset(obs_out=self._obs, **kw)
        self.episode = self.env.episode
        self._sync_copy(False)
        self.done = False
        self.reset_obs = self._host_f.numpy()[:self.n * self.N * self.F].reshape(self.n, self.N, self.F).copy()
        self.reset_taken = np.zeros(self.n, dtype=bool)
        return self.reset_obs

    def reset_one(self, i):
        """RLlib's per-env reset: the first call after the batch's episode ended resets the batch."""
        i = int(i)
        if not 0 <= i < self.n:
            raise IndexError("env index %d outside the batch of %d" % (i, self.n))
        if self.reset_obs is not None and not self.reset_taken[i]:
            self.reset_taken[i] = True          # this env's row of the batched reset already run
            return self.reset_obs[i]
        # a new batched reset: before the first episode, after the batch's episode ended, or a whole
        # second round of resets at period 0; never in the middle of an episode
        fresh_round = self.env.period == 0 and self.reset_taken is not None and bool(self.reset_taken.all())
        if self.episode >= 0 and not self.done and not fresh_round:
            raise RuntimeError("env %d: the batch steps in lockstep (one shared period); an env can be reset "
                               "only when the batch's episode has ended" % i)
        self.reset_all()
        self.reset_taken[i] = True
        return self.reset_obs[i]

    def step(self, actions):
        """actions [n, N] (host, float64 after np.asarray) -> host (obs [n,N,F], reward [n] or [n,N],
        info dict of [n,N] arrays or None, period after the step)."""
        if self.done:
            raise RuntimeError("the batch's episode has ended: reset first (IMENV_E_DONE)")
        t = self.env.period
        self._host_a.numpy()[:] = np.asarray(actions, dtype=np.float64).reshape(self.n, self.N)
        self._dev_a.copy_(self._host_a, non_blocking=True)
        _, _, done, _ = self.env.step(self._dev_a, obs_out=self._obs, reward_out=self._rew,
                                      info_out=self._info if self.info else None)
        self._sync_copy(self.info)
        self.reset_obs = None       # a reset_at now would be mid-episode (refused unless done)
        self.done = done
        n, N, F = self.n, self.N, self.F
        hf, hi = self._host_f.numpy(), self._host_i.numpy()
        obs = hf[:n * N * F].reshape(n, N, F)
        rew = hf[n * N * F:n * N * F + n * self.nr].reshape((n, N) if self.nr == N else (n,))
        info = None
        if self.info:
            iv = lambda j: hi[j * n * N:(j + 1) * n * N].reshape(n, N).astype(np.float64)
            # profit is copied out of the host mirror like the others (astype copies): the mirror is
            # rewritten by the next step, and RLlib keeps infos in its sample batches (IM_env.py:350
            # hands out a fresh array per step)
            info = dict(order=iv(0), demand=iv(1), acquisition=iv(2), ship=iv(3),
                        profit=hf[n * N * F + n * self.nr:].reshape(n, N).copy())
        return obs, rew, info, t

    def close(self):
        self.env.close()


class InvVectorEnv(_VectorEnv):
    """RLlib VectorEnv of ``num_envs`` single-agent envs (kind "IM": InvManagement, IM_env.py; "IM_div":
    InvManagementDiv, IM_div_env.py) stepped by one kernel launch per vector_step.

        register_env("InventoryManagement", lambda cfg: InvVectorEnv("IM", cfg, num_envs=64))
    """

    def __init__(self, kind, config, num_envs, device=None, env_offset=None, info=True, episode_inputs=None):
        if kind not in ("IM", "IM_div"):
            raise ValueError("InvVectorEnv is for the single-agent classes (IM, IM_div); use InvMultiAgentBaseEnv")
        self._b = _Batch(kind, config, num_envs, device, env_offset, info, episode_inputs)
        self.num_envs = self._b.n
        self.observation_space = self._b.observation_space
        self.action_space = self._b.action_space

    def vector_reset(self):
        """Every env's period-0 observation (IM_env.py:164-229): a list of num_envs [N, F] arrays."""
        obs = self._b.reset_all()
        self._b.reset_taken[:] = True
        return [obs[i] for i in range(self.num_envs)]

    def reset_at(self, index=None):
        return self._b.reset_one(0 if index is None else index)

    def vector_step(self, actions):
        """IM_env.py:287-360 for every env: actions = num_envs action arrays ([N] each) -> lists of obs
        ([N, F]), rewards (float), dones (bool) and infos (period, demand, ship, acquisition, profit)."""
        obs, rew, info, t = self._b.step(actions)
        n = self.num_envs
        done = self._b.done
        obs_l = list(obs.copy())                # per-env views of one fresh copy (the host mirror is reused)
        rew_l = rew.tolist()
        if info is not None:
            dem, shp, acq, pro = (list(info[k]) for k in ("demand", "ship", "acquisition", "profit"))
            infos = [{"period": t, "demand": dem[i], "ship": shp[i], "acquisition": acq[i], "profit": pro[i]}
                     for i in range(n)]
        else:
            infos = [{} for _ in range(n)]
        return obs_l, rew_l, [done] * n, infos

    def get_unwrapped(self):
        return []       # no per-env gym objects: the batch lives in HBM

    def get_sub_environments(self):
        return []

    def try_render_at(self, index=None):
        return None

    def close(self):
        self._b.close()


class InvMultiAgentBaseEnv(_BaseEnv):
    """RLlib BaseEnv of ``num_envs`` multi-agent envs (kind "MAIM": MultiAgentInvManagement, MAIM_env.py;
    "MAIM_div": MultiAgentInvManagementDiv, MAIM_div_env.py) stepped by one kernel launch per
    send_actions; agent ids stage_i / node_i.

        register_env("MultiAgentInventoryManagement",
                     lambda cfg: InvMultiAgentBaseEnv("MAIM", cfg, num_envs=64))
    """

    def __init__(self, kind, config, num_envs, device=None, env_offset=None, info=True, episode_inputs=None):
        if kind not in ("MAIM", "MAIM_div"):
            raise ValueError("InvMultiAgentBaseEnv is for the multi-agent classes (MAIM, MAIM_div); use InvVectorEnv")
        self._b = _Batch(kind, config, num_envs, device, env_offset, info, episode_inputs)
        self.num_envs = self._b.n
        prefix = "stage_" if kind == "MAIM" else "node_"
        self.agent_ids = [prefix + str(i) for i in range(self._b.N)]
        self.observation_space = self._b.observation_space     # one agent's
        self.action_space = self._b.action_space
        self._obs = None          # per env: {agent: obs} ready to release (None: not initialised yet)
        self._last_rew = [dict() for _ in range(self.num_envs)]
        self._last_done = [dict() for _ in range(self.num_envs)]
        self._last_info = [dict() for _ in range(self.num_envs)]
        self._dones = set()

    # RLlib's _MultiAgentEnvState.reset for env i, from the batch's reset row
    def _env_reset(self, i, row):
        obs = {ag: row[k].copy() for k, ag in enumerate(self.agent_ids)}
        self._obs[i] = obs
        self._last_rew[i] = {ag: None for ag in self.agent_ids}
        self._last_done[i] = {ag: False for ag in self.agent_ids}
        self._last_done[i]["__all__"] = False
        self._last_info[i] = {ag: {} for ag in self.agent_ids}
        return obs

    def poll(self):
        """(obs, rewards, dones, infos, off_policy_actions), each {env_id: {agent_id: value}}, for the
        envs with a new observation (all of them after a step or the first poll)."""
        if self._obs is None:               # first poll: every env resets (one batched reset)
            rows = self._b.reset_all()
            self._b.reset_taken[:] = True
            self._obs = [None] * self.num_envs
            for i in range(self.num_envs):
                self._env_reset(i, rows[i])
        obs_d, rew_d, done_d, info_d = {}, {}, {}, {}
        for i in range(self.num_envs):
            obs = self._obs[i]
            if obs is None:
                obs_d[i], rew_d[i], done_d[i], info_d[i] = {}, {}, {"__all__": False}, {}
                continue
            lr, ld, li = self._last_rew[i], self._last_done[i], self._last_info[i]
            if ld.get("__all__", False):        # episode over: release everything
                rew, done, info = lr, ld, li
                self._last_rew[i], self._last_done[i], self._last_info[i] = {}, {}, {}
                self._obs[i] = {}
            elif obs:
                # the observation holds every agent of the env, so every pending agent entry is
                # released: the pending dicts themselves are handed out and start over empty
                rew, done, info = lr, ld, li
                done["__all__"] = False
                self._last_rew[i], self._last_done[i], self._last_info[i] = {}, {}, {}
                self._obs[i] = {}            # released once: a second poll before send_actions gets none
            else:
                rew, done, info = {}, {"__all__": False}, {}
            self._last_done[i]["__all__"] = False
            obs_d[i], rew_d[i], done_d[i], info_d[i] = obs, rew, done, info
        return obs_d, rew_d, done_d, info_d, {}

    def send_actions(self, action_dict):
        """{env_id: {agent_id: action}} for every env of the batch (lockstep: one step of all)."""
        n = self.num_envs
        for env_id in action_dict:
            if env_id in self._dones:
                raise ValueError("Env {} is already done".format(env_id))
        if len(action_dict) != n:
            raise ValueError("the batch steps its %d envs in lockstep: actions for every env are needed (got %d)"
                             % (n, len(action_dict)))
        ids, N = self.agent_ids, self._b.N
        try:
            flat = [action_dict[i][ag] for i in range(n) for ag in ids]
        except KeyError as e:
            raise ValueError("actions for env ids 0..%d and agents %s are needed (missing %r)" % (n - 1, ids, e.args[0]))
        try:
            act = np.asarray(flat, dtype=np.float64).reshape(n, N)     # one scalar or 1-element array each
        except ValueError:
            act = np.array([float(np.asarray(x, dtype=np.float64).reshape(-1)[0]) for x in flat]).reshape(n, N)
        obs, rew, info, t = self._b.step(act)
        done = self._b.done
        period = t + 1
        rows = list(obs.copy().reshape(n * N, -1))     # per-agent views of one fresh copy
        rv = list(rew.ravel())                         # np.float64 scalars: [n] shared or [n, N] per agent
        indep = len(rv) == n * N
        if info is not None:            # one info dict per (env, agent), env-major
            infs = [{"period": period, "demand": d, "ship": s, "acquisition": a, "actual order": o, "profit": p}
                    for d, s, a, o, p in zip(*(info[k].ravel() for k in ("demand", "ship", "acquisition", "order",
                                                                          "profit")))]
        for i in range(n):
            b = i * N
            o = dict(zip(ids, rows[b:b + N]))
            r = dict(zip(ids, rv[b:b + N])) if indep else dict.fromkeys(ids, rv[i])
            if info is not None:
                inf = dict(zip(ids, infs[b:b + N]))
            else:
                inf = {ag: {} for ag in ids}
            # RLlib's _MultiAgentEnvState.observe
            self._obs[i] = o
            lr = self._last_rew[i]
            if lr:
                for ag, v in r.items():
                    p = lr.get(ag)
                    lr[ag] = v if p is None else p + v
            else:
                self._last_rew[i] = r
            ld = self._last_done[i]
            ld["__all__"] = (ld["__all__"] or done) if "__all__" in ld else done
            self._last_info[i] = inf
            if done:
                self._dones.add(i)

    def try_reset(self, env_id=None):
        """Reset env env_id (RLlib calls it per env once its episode is done): {agent_id: obs}."""
        i = 0 if env_id is None else int(env_id)
        row = self._b.reset_one(i)
        obs = self._env_reset(i, row)
        self._dones.discard(i)
        return obs

    def get_unwrapped(self):
        return []

    def get_sub_environments(self):
        return []

    def try_render(self, env_id=None):
        return None

    def stop(self):
        self._b.close()

    def close(self):
        self._b.close()


__all__ = ["InvVectorEnv", "InvMultiAgentBaseEnv"]

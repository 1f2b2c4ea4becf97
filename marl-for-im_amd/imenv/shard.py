"""Multi-GPU sharding: one process per GPU, each owning a contiguous range of global env ids.

Envs are independent (no cross-env term anywhere in step()), so the data path
has no collective: rank r steps envs [offset_r, offset_r + n_r) on its own GPU, and every
random draw is keyed by the GLOBAL env id (Philox counter, imenv.h), so trajectories do not
depend on the number of ranks. The only exchange is optional: gathering each step's observations
and rewards to every rank (a centralised learner), one RCCL all-gather per step.
"""
import torch
import torch.distributed as dist


def shard_range(total_envs, world_size, rank):
    """(offset, count) of rank's contiguous share of total_envs; the first total % world ranks get one
    more env."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError("rank %d outside world of %d" % (rank, world_size))
    base, extra = divmod(int(total_envs), int(world_size))
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def weak_offset(n_per_rank, rank):
    """Global id of rank's first env when every rank owns n_per_rank envs (weak scaling)."""
    return int(rank) * int(n_per_rank)


class StepGather:
    """All-gathers one step's obs [n, N, F] and reward [n] / [n, N] from every rank (equal n).

    Buffers are allocated once; NCCL (RCCL) uses all_gather_into_tensor straight into them, other
    backends (gloo, CPU tests) all_gather a list and copy.
    """

    def __init__(self, obs_like, reward_like, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.obs = torch.empty((self.world * obs_like.shape[0],) + tuple(obs_like.shape[1:]), dtype=obs_like.dtype,
                               device=obs_like.device)
        self.reward = torch.empty((self.world * reward_like.shape[0],) + tuple(reward_like.shape[1:]),
                                  dtype=reward_like.dtype, device=reward_like.device)
        self._into = dist.get_backend(group) == "nccl"

    def _one(self, out, x):
        if self._into:
            dist.all_gather_into_tensor(out, x.contiguous(), group=self.group)
        else:
            dist.all_gather(list(out.chunk(self.world, dim=0)), x.contiguous(), group=self.group)   # views

    def __call__(self, obs, reward):
        self._one(self.obs, obs)
        self._one(self.reward, reward)
        return self.obs, self.reward

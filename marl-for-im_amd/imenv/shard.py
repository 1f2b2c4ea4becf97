"""Multi-GPU sharding: one process per GPU, each owning a contiguous range of global env ids.

Envs are independent (no cross-env term anywhere in step()), so the data path
has no collective: rank r steps envs [offset_r, offset_r + n_r) on its own GPU, and every
random draw is keyed by the GLOBAL env id (Philox counter, imenv.h), so trajectories do not
depend on the number of ranks. The only exchange is optional: gathering observations and rewards
to every rank (a centralised learner).

The gather packs every field of one exchange into ONE byte buffer, so one RCCL all-gather moves
them all. The env writes straight into that buffer (``obs_out`` / ``reward_out`` views), so there is
no packing copy. xGMI links are point to point (7 links per GPU), so a ring all-gather is bound per
link. Fewer, larger collectives therefore win:
- ``StepGather``: one collective per step, double-buffered. The collective of step t overlaps step
  t+1 on RCCL's stream (``async_op``); the send buffer is reused only after that collective completes.
- ``EpisodeGather``: one collective per episode over the whole [T+1, n, ...] rollout. It moves 30x
  the bytes per call and makes 30x fewer calls.
The evaluation harness's statistics over sharded test episodes need one small collective:
``global_metrics_stats`` all-gathers each rank's (mean, std, count) per metric column and merges
them (Chan et al.), so the mean / std are those of all envs on all ranks.
"""
import torch
import torch.distributed as dist

_ALIGN = 256     # every field starts on a 256-byte boundary of the packed buffer


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


class PackedGather:
    """All-gather of several tensors (equal shapes on every rank) as one packed byte buffer.

    fields: [(shape, dtype), ...]. ``send(k)`` gives the fields of send buffer k as contiguous views
    to write into (VectorInvEnv.step(obs_out=..., reward_out=...) accepts them). ``gathered(k)`` gives
    every field of receive buffer k as a [world, *shape] view. ``start(k)`` launches the collective of
    buffer k and ``wait(k)`` orders the current stream after it.
    """

    def __init__(self, fields, device, group=None, buffers=1):
        self.group = group
        self.world = dist.get_world_size(group)
        self.fields = [(tuple(int(s) for s in shape), dtype) for shape, dtype in fields]
        self.offsets, off = [], 0
        for shape, dtype in self.fields:
            self.offsets.append(off)
            nbytes = torch.Size(shape).numel() * torch.empty((), dtype=dtype).element_size()
            off += (nbytes + _ALIGN - 1) // _ALIGN * _ALIGN
        self.chunk = off
        self.device = torch.device(device)
        # an all-gather needs one send size on every rank: RCCL given different counts hangs or corrupts
        # memory instead of raising, so the sizes are compared first (one collective of equal shape)
        if self.world > 1:
            sz = torch.tensor([off, -off], dtype=torch.int64, device=self.device)
            dist.all_reduce(sz, op=dist.ReduceOp.MAX, group=group)
            if int(sz[0]) != off or -int(sz[1]) != off:
                raise ValueError("PackedGather: the ranks' send buffers differ in size (this rank %d bytes, "
                                 "largest %d, smallest %d): shard the envs evenly" % (off, int(sz[0]), -int(sz[1])))
        self._send = [torch.empty(self.chunk, dtype=torch.uint8, device=self.device) for _ in range(buffers)]
        self._recv = [torch.empty(self.world * self.chunk, dtype=torch.uint8, device=self.device)
                      for _ in range(buffers)]
        self._work = [None] * buffers
        self._into = dist.get_backend(group) == "nccl"
        self._kept = None       # completed collectives, kept for timing (keep_works)
        # the field views of every buffer, made once: a per-step loop then pays no torch view ops
        # (about a dozen per step otherwise, each a few microseconds of host time)
        self._send_views = [[self._field(b, j) for j in range(len(self.fields))] for b in self._send]
        self._recv_views = [[self._field(b, j, lead=(self.world,)) for j in range(len(self.fields))]
                            for b in self._recv]
        self._recv_lists = [list(b.chunk(self.world)) for b in self._recv]

    def _field(self, buf, j, lead=()):
        shape, dtype = self.fields[j]
        nbytes = torch.Size(shape).numel() * torch.empty((), dtype=dtype).element_size()
        o = self.offsets[j]
        if not lead:
            return buf[o:o + nbytes].view(dtype).view(shape)
        rows = buf.view(self.world, self.chunk)[:, o:o + nbytes]     # [world, nbytes], rows contiguous
        return rows.view(dtype).view((self.world,) + shape)

    def send(self, k=0):
        return list(self._send_views[k])

    def gathered(self, k=0):
        return list(self._recv_views[k])

    def start(self, k=0):
        """Launch the all-gather of send buffer k (async: RCCL's stream waits for the work already
        queued on the current stream, the current stream does not wait for the collective)."""
        self.wait(k)         # a previous collective on these buffers must be complete first
        if self._into:
            self._work[k] = dist.all_gather_into_tensor(self._recv[k], self._send[k], group=self.group,
                                                        async_op=True)
        else:
            self._work[k] = dist.all_gather(self._recv_lists[k], self._send[k], group=self.group, async_op=True)

    def wait(self, k=0):
        w = self._work[k]
        if w is not None:
            w.wait()          # NCCL: a stream dependency, not a host block
            self._work[k] = None
            if self._kept is not None:
                self._kept.append(w)

    def keep_works(self, on):
        """Start (on=True) or stop keeping every collective's Work object once it has been waited for
        (bench.py reads each one's own duration, Work._get_duration, with TORCH_NCCL_ENABLE_TIMING=1).
        Returns the Works kept so far."""
        kept = self._kept or []
        self._kept = [] if on else None
        return kept

    def __call__(self, *tensors, k=0):
        """Copy tensors into send buffer k, gather synchronously, return the [world, ...] views."""
        self.wait(k)
        for dst, src in zip(self.send(k), tensors):
            dst.copy_(src)
        self.start(k)
        self.wait(k)
        return self.gathered(k)


class StepGather(PackedGather):
    """One step's obs [n, N, F] and reward [n] / [n, N] from every rank, double-buffered: the env of
    step t writes into ``obs_out(t)`` / ``reward_out(t)`` (buffer t % 2), ``start(t)`` launches the
    gather, which overlaps step t+1; ``result(t)`` waits for it and returns (obs [world*n, N, F],
    reward [world*n, ...]) views."""

    def __init__(self, obs_like, reward_like, group=None, buffers=2):
        super().__init__([(obs_like.shape, obs_like.dtype), (reward_like.shape, reward_like.dtype)],
                         obs_like.device, group, buffers)
        self.nbuf = buffers
        # result()'s [world * n, ...] tensors: cached where flatten is a view of the receive buffer
        # (world 1), made per call where it is a copy (world > 1: the ranks' rows sit a packed chunk apart)
        self._flat = []
        for views in self._recv_views:
            f = tuple(v.flatten(0, 1) for v in views)
            self._flat.append(f if all(a.data_ptr() == v.data_ptr() for a, v in zip(f, views)) else None)

    def obs_out(self, t):
        """Send view for step t's obs. Orders the current stream after the collective that last read
        this buffer (step t - nbuf), so the env cannot overwrite it while it is in flight."""
        self.wait(t % self.nbuf)
        return self._send_views[t % self.nbuf][0]

    def reward_out(self, t):
        self.wait(t % self.nbuf)
        return self._send_views[t % self.nbuf][1]

    def start(self, t=0):
        super().start(t % self.nbuf)

    def result(self, t):
        self.wait(t % self.nbuf)
        f = self._flat[t % self.nbuf]
        if f is not None:
            return f
        o, r = self._recv_views[t % self.nbuf]
        return o.flatten(0, 1), r.flatten(0, 1)

    def __call__(self, obs, reward):
        """Compatibility: copy one step's obs / reward in and gather synchronously (buffer 0)."""
        o, r = PackedGather.__call__(self, obs, reward, k=0)
        return o.flatten(0, 1), r.flatten(0, 1)


class EpisodeGather(PackedGather):
    """A whole episode's rollout (obs [T+1, n, N, F], rewards [T, n(, N)]) in one collective: the env
    writes every period into ``obs`` / ``rewards`` (views of the send buffer); ``start()`` after the
    last step; ``result()`` -> [world, T+1, n, N, F] and [world, T, n(, N)] views."""

    def __init__(self, env, group=None, obs_dtype=torch.float32):
        T, n, N, F = env.T, env.n, env.N, env.F
        super().__init__([((T + 1, n, N, F), obs_dtype), ((T,) + tuple(env.reward_shape()), torch.float64)],
                         env.device, group, 1)
        self.obs, self.rewards = self.send(0)

    def result(self):
        self.wait(0)
        return self.gathered(0)


def merge_column_stats(stats, counts):
    """Per-rank np.mean / np.std (population) of the same columns -> those of the union of the rows.

    stats: [W, C, 2] (mean, std) per rank; counts: [W] rows per rank. Chan et al.'s pairwise update
    in float64: M2 = sum_r (n_r std_r^2 + n_r (mean_r - mean)^2), mean = sum_r n_r mean_r / n."""
    stats = torch.as_tensor(stats, dtype=torch.float64)
    n_r = torch.as_tensor(counts, dtype=torch.float64).reshape(-1, 1)
    n = n_r.sum()
    mean = (n_r * stats[..., 0]).sum(0) / n
    m2 = (n_r * stats[..., 1] ** 2 + n_r * (stats[..., 0] - mean) ** 2).sum(0)
    return torch.stack([mean, torch.sqrt(m2 / n)], dim=-1)


def gather_column_stats(local_stats, count, group=None):
    """All-gather every rank's [C, 2] (mean, std) and row count (one collective of C*2+1 doubles) and
    merge them: the evaluation harness's mean / std over the envs of all ranks
    (inv_management.py:608-643 over the whole test set, when the test episodes are sharded)."""
    ls = local_stats.to(torch.float64)
    buf = torch.cat([ls.reshape(-1), torch.tensor([float(count)], dtype=torch.float64, device=ls.device)])
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        out = torch.empty(world * buf.numel(), dtype=torch.float64, device=ls.device)
        dist.all_gather_into_tensor(out, buf, group=group)
        rows = out.view(world, -1)
    else:
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=group)
        rows = torch.stack(parts)
    rows = rows.cpu()
    C = ls.shape[0]
    return merge_column_stats(rows[:, :-1].reshape(world, C, 2), rows[:, -1])


def global_metrics_stats(env, group=None):
    """np.mean / np.std of every evaluation-harness metric column over the envs of every rank
    (VectorInvEnv.metrics_stats on each rank, then gather_column_stats)."""
    return gather_column_stats(env.metrics_stats(), env.n, group)

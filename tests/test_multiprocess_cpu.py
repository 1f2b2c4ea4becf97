"""World-size-2 gloo runs of the sharded path on CPU.

Each rank owns a contiguous range of global env ids (imenv.shard), draws demand keyed by the
GLOBAL id (the oracle's Philox twin of the kernel's draws), steps its shard and all-gathers every
step's obs and reward with imenv.shard.StepGather (the same helper bench.py --gather uses with
RCCL). Rank 0's gathered trajectory must equal one single-process run over all envs, which is what
makes the GPU count invisible in the results.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from imenv.shard import StepGather, gather_column_stats, merge_column_stats, shard_range, weak_offset

C2 = dict(num_stages=4, num_periods=30, init_inv=np.ones(4) * 10, inv_target=np.zeros(4),
          inv_max=np.ones(4) * 30, price=np.array([5, 4, 3, 2, 1]),
          stock_cost=np.array([0.35, 0.3, 0.4, 0.2]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.9]),
          delay=np.array([1, 2, 3, 1]), demand_dist="poisson", mu=5, seed=52, independent=False)
C4 = dict(num_nodes=4, connections={0: [1], 1: [2, 3], 2: [], 3: []}, num_periods=30,
          init_inv=np.ones(4) * 10, inv_target=np.zeros(4), inv_max=np.ones(4) * 30,
          stock_cost=np.array([0.35, 0.3, 0.4, 0.4]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.6]),
          delay=np.array([1, 2, 1, 1]), demand_dist="poisson", mu=5, seed=52, time_dependency=True,
          prev_demand=True, independent=True)
N_TOTAL = 96


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _actions(kind, n_total, T):
    rs = np.random.RandomState(11)
    return rs.uniform(-1.1, 1.1, size=(T, n_total, 4)).astype(np.float32).astype(np.float64)


def _rollout(kind, cfg, offset, count, acts, gather=None):
    from oracle.im_oracle import OracleEnv
    env = OracleEnv(kind, cfg, n_envs=count)
    obs_all, rew_all = [], []
    for ep in range(2):
        env.reset(rng=dict(seed=52, episode=ep, env_offset=offset, dist="poisson", mu=5))
        for t in range(30):
            obs, rew, _, _ = env.step(acts[t, offset:offset + count])
            o, r = torch.from_numpy(np.ascontiguousarray(obs)), torch.from_numpy(np.ascontiguousarray(rew))
            if gather is not None:
                o, r = gather(o, r)
            obs_all.append(o.clone())
            rew_all.append(r.clone())
    return torch.stack(obs_all), torch.stack(rew_all)


def _worker(rank, world, port, kind, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = C2 if kind == "MAIM" else C4
        offset, count = shard_range(N_TOTAL, world, rank)
        acts = _actions(kind, N_TOTAL, 30)
        from oracle.im_oracle import OracleEnv
        probe = OracleEnv(kind, cfg, n_envs=count)
        o0 = probe.reset(rng=dict(seed=52, episode=0, env_offset=offset, dist="poisson", mu=5))
        r_shape = (count,) + ((4,) if kind == "MAIM_div" else ())
        g = StepGather(torch.zeros((count,) + o0.shape[1:], dtype=torch.float64),
                       torch.zeros(r_shape, dtype=torch.float64))
        obs, rew = _rollout(kind, cfg, offset, count, acts, gather=g)
        # timing contract of bench.py: max over ranks
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            torch.save(dict(obs=obs, rew=rew, tmax=t), out_path)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["MAIM", "MAIM_div"])
def test_two_rank_gather_equals_single_run(kind, tmp_path):
    out = str(tmp_path / "rank0.pt")
    mp.spawn(_worker, args=(2, _free_port(), kind, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    cfg = C2 if kind == "MAIM" else C4
    ref_obs, ref_rew = _rollout(kind, cfg, 0, N_TOTAL, _actions(kind, N_TOTAL, 30))
    assert torch.equal(got["obs"], ref_obs)
    assert torch.equal(got["rew"], ref_rew)
    assert got["tmax"].item() == 2.0


def test_shard_range_partitions_ids():
    for total in (1, 7, 96, 1 << 20):
        for world in (1, 2, 3, 8):
            if total < world:
                continue
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            assert sum(c for _, c in spans) == total
            for (o1, c1), (o2, _) in zip(spans, spans[1:]):
                assert o1 + c1 == o2
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    assert weak_offset(1 << 20, 3) == 3 << 20


class _EnvShape:
    """The attributes EpisodeGather reads from a VectorInvEnv (CPU stand-in for the gloo test)."""
    def __init__(self, T, n, N, F, independent):
        self.T, self.n, self.N, self.F = T, n, N, F
        self.device = torch.device("cpu")
        self._ind = independent

    def reward_shape(self):
        return (self.n, self.N) if self._ind else (self.n,)


def _packed_worker(rank, world, port, out_path):
    from imenv.shard import EpisodeGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, N, F, T = 5, 4, 3, 30
        # per-step, double-buffered: write step t into buffer t % 2 while step t-1's gather is in flight
        g = StepGather(torch.zeros((n, N, F)), torch.zeros(n, dtype=torch.float64))
        g.keep_works(True)       # bench.py --gather times each collective from its kept Work
        steps = []
        for t in range(6):
            g.obs_out(t).copy_(torch.full((n, N, F), 100.0 * rank + t))
            g.reward_out(t).copy_(torch.arange(n, dtype=torch.float64) + 1000 * rank + t)
            g.start(t)
            if t >= 1:
                steps.append([x.clone() for x in g.result(t - 1)])
        steps.append([x.clone() for x in g.result(5)])
        kept = g.keep_works(False)
        assert len(kept) == 6 and all(w.is_completed() for w in kept), len(kept)
        assert g.keep_works(False) == []
        # per-episode: one collective over the whole rollout, independent (per-agent) rewards
        eg = EpisodeGather(_EnvShape(T, n, N, F, independent=True))
        eg.obs.copy_(torch.arange((T + 1) * n * N * F, dtype=torch.float32).view(T + 1, n, N, F) + rank)
        eg.rewards.copy_(torch.full((T, n, N), -1.0 - rank, dtype=torch.float64))
        eg.start()
        eo, er = eg.result()
        if rank == 0:
            torch.save(dict(steps=steps, eo=eo.clone(), er=er.clone()), out_path)
    finally:
        dist.destroy_process_group()


def test_packed_step_and_episode_gathers(tmp_path):
    out = str(tmp_path / "packed.pt")
    mp.spawn(_packed_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    n, N, F, T = 5, 4, 3, 30
    for t, (o, r) in enumerate(got["steps"]):
        assert o.shape == (2 * n, N, F) and r.shape == (2 * n,)
        for rank in range(2):
            assert torch.equal(o[rank * n:(rank + 1) * n], torch.full((n, N, F), 100.0 * rank + t))
            assert torch.equal(r[rank * n:(rank + 1) * n], torch.arange(n, dtype=torch.float64) + 1000 * rank + t)
    base = torch.arange((T + 1) * n * N * F, dtype=torch.float32).view(T + 1, n, N, F)
    assert got["eo"].shape == (2, T + 1, n, N, F) and got["er"].shape == (2, T, n, N)
    for rank in range(2):
        assert torch.equal(got["eo"][rank], base + rank)
        assert torch.equal(got["er"][rank], torch.full((T, n, N), -1.0 - rank, dtype=torch.float64))


def _stats_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x = np.random.RandomState(7).normal(10, 50, size=(1001, 8))       # every rank builds the same table
        offset, count = shard_range(len(x), world, rank)
        mine = torch.from_numpy(x[offset:offset + count])
        local = torch.stack([mine.mean(0), mine.std(0, unbiased=False)], dim=-1)
        got = gather_column_stats(local, count)
        if rank == 0:
            torch.save(dict(got=got), out_path)
    finally:
        dist.destroy_process_group()


def test_metric_stats_over_ranks(tmp_path):
    """The harness's np.mean / np.std over the envs of all ranks from per-rank stats (Chan merge)."""
    out = str(tmp_path / "stats.pt")
    mp.spawn(_stats_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)["got"].numpy()
    x = np.random.RandomState(7).normal(10, 50, size=(1001, 8))
    np.testing.assert_allclose(got[:, 0], x.mean(0), rtol=1e-12)
    np.testing.assert_allclose(got[:, 1], x.std(0), rtol=1e-12)
    # merging a single rank is the identity; empty-free uneven splits
    one = merge_column_stats(torch.tensor([[[3.0, 2.0]]]), [5])
    assert torch.allclose(one, torch.tensor([[3.0, 2.0]], dtype=torch.float64))


def _uneven_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 5 + rank          # shard_range of an odd total: the first rank holds one env more
        try:
            StepGather(torch.zeros((n, 4, 3)), torch.zeros(n, dtype=torch.float64))
            msg = None
        except ValueError as e:
            msg = str(e)
        torch.save(dict(msg=msg), out_path + str(rank))
    finally:
        dist.destroy_process_group()


def test_uneven_shards_are_refused_before_any_gather(tmp_path):
    """Ranks whose send buffers differ (uneven shards) are refused on every rank at construction, before an
    all-gather could be handed different counts (RCCL: undefined behaviour, not an exception)."""
    out = str(tmp_path / "uneven.pt")
    mp.spawn(_uneven_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        msg = torch.load(out + str(r), weights_only=True)["msg"]
        assert msg is not None and "differ in size" in msg

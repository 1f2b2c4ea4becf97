"""HIP graph capture of whole episodes (reset + T steps) through the C ABI.

Launch-bound batches (the step kernel's back-to-back dispatch costs ~4 us below ~2^17 envs) replay a
captured episode instead of launching 31 kernels from the host. Every replay must equal an eager
episode: the reset kernel advances the device-resident episode counter, so each replay draws the
next episode's demand, and the captured step launches carry their period t as a kernel argument.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

C2 = dict(num_stages=4, num_periods=30, init_inv=np.ones(4) * 10, inv_target=np.zeros(4),
          inv_max=np.ones(4) * 30, price=np.array([5, 4, 3, 2, 1]),
          stock_cost=np.array([0.35, 0.3, 0.4, 0.2]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.9]),
          delay=np.array([1, 2, 3, 1]), demand_dist="poisson", mu=5, seed=52, independent=False)
C4 = dict(num_nodes=4, connections={0: [1], 1: [2, 3], 2: [], 3: []}, num_periods=30,
          init_inv=np.ones(4) * 10, inv_target=np.zeros(4), inv_max=np.ones(4) * 30,
          stock_cost=np.array([0.35, 0.3, 0.4, 0.4]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.6]),
          delay=np.array([1, 2, 1, 1]), demand_dist="poisson", mu=5, seed=52, time_dependency=True,
          prev_demand=True, independent=False)


@pytest.mark.parametrize("kind,cfg", [("MAIM", C2), ("MAIM_div", C4)])
def test_graph_replay_equals_eager_episodes(kind, cfg):
    from imenv import VectorInvEnv
    n = 4096
    g_env = VectorInvEnv(kind, cfg, n_envs=n, device=DEV)
    e_env = VectorInvEnv(kind, cfg, n_envs=n, device=DEV)
    T, N, F = g_env.T, g_env.N, g_env.F
    gen = torch.Generator(device=DEV)
    gen.manual_seed(3)
    act = torch.rand((T, n, N), generator=gen, device=DEV) * 2 - 1
    obs = torch.empty((T + 1, n, N, F), dtype=torch.float32, device=DEV)
    rew = torch.empty((T, n), dtype=torch.float64, device=DEV)
    # episode 0 eagerly on both (the first step of a flag combination compiles its kernel)
    for env in (g_env, e_env):
        env.reset(obs_out=obs[0])
        for t in range(T):
            env.step(act[t], obs_out=obs[t + 1], reward_out=rew[t])
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        g_env.reset(obs_out=obs[0])
        for t in range(T):
            g_env.step(act[t], obs_out=obs[t + 1], reward_out=rew[t])
    assert g_env.kernel_info().startswith("jit:"), g_env.kernel_info()
    e_obs = torch.empty_like(obs)
    e_rew = torch.empty_like(rew)
    for replay in range(3):                      # replays = episodes 1, 2, 3
        graph.replay()
        e_env.reset(obs_out=e_obs[0])
        for t in range(T):
            e_env.step(act[t], obs_out=e_obs[t + 1], reward_out=e_rew[t])
        torch.cuda.synchronize()
        assert torch.equal(obs, e_obs), "replay %d obs" % replay
        assert torch.equal(rew, e_rew), "replay %d reward" % replay
    g_env.close()
    e_env.close()


def test_graph_captures_policy_and_env_together():
    """A torch policy and the env step in one captured episode (the launch-bound inner loop of a
    trainer's sampler): replay == the same loop run eagerly."""
    from imenv import VectorInvEnv
    n = 2048
    torch.manual_seed(0)
    pol = torch.nn.Sequential(torch.nn.Linear(3, 16), torch.nn.Tanh(), torch.nn.Linear(16, 1), torch.nn.Tanh()).to(DEV)
    envs = [VectorInvEnv("MAIM", C2, n_envs=n, device=DEV) for _ in range(2)]
    T, N, F = envs[0].T, envs[0].N, envs[0].F
    bufs = [(torch.empty((T + 1, n, N, F), device=DEV), torch.empty((T, n, N), device=DEV),
             torch.empty((T, n), dtype=torch.float64, device=DEV)) for _ in range(2)]

    def episode(env, buf):
        obs, act, rew = buf
        env.reset(obs_out=obs[0])
        for t in range(T):
            act[t].copy_(pol(obs[t]).squeeze(-1))                       # per-agent action from its own obs
            env.step(act[t], obs_out=obs[t + 1], reward_out=rew[t])

    with torch.no_grad():
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):                                      # warm-up (compiles, allocates)
            for env, buf in zip(envs, bufs):
                episode(env, buf)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            episode(envs[0], bufs[0])
        for _ in range(2):
            g.replay()
            episode(envs[1], bufs[1])
            torch.cuda.synchronize()
            for x, y in zip(bufs[0], bufs[1]):
                assert torch.equal(x, y)
    for env in envs:
        env.close()


def test_mixed_eager_and_replayed_episodes():
    """Eager episodes, graph replays and explicit episode numbers interleaved on one handle: every
    episode equals the same episode run eagerly on a second handle (the reset kernel advances the
    device episode word in a replay exactly as in an eager reset, and an explicit number sets it)."""
    from imenv import VectorInvEnv
    n = 2048
    a_env = VectorInvEnv("MAIM", C2, n_envs=n, device=DEV)
    b_env = VectorInvEnv("MAIM", C2, n_envs=n, device=DEV)
    T, N, F = a_env.T, a_env.N, a_env.F
    gen = torch.Generator(device=DEV)
    gen.manual_seed(5)
    act = torch.rand((T, n, N), generator=gen, device=DEV) * 2 - 1
    bufs = [(torch.empty((T + 1, n, N, F), device=DEV), torch.empty((T, n), dtype=torch.float64, device=DEV))
            for _ in range(2)]

    def episode(env, buf, ep=None):
        obs, rew = buf
        env.reset(obs_out=obs[0], episode=ep)
        for t in range(T):
            env.step(act[t], obs_out=obs[t + 1], reward_out=rew[t])

    def same(tag):
        torch.cuda.synchronize()
        assert torch.equal(bufs[0][0], bufs[1][0]) and torch.equal(bufs[0][1], bufs[1][1]), tag

    episode(a_env, bufs[0]); episode(b_env, bufs[1]); same("eager episode 0")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        episode(a_env, bufs[0])
    assert a_env.kernel_info().startswith("jit:"), a_env.kernel_info()
    for k in (1, 2):                                   # replays: episodes 1, 2
        g.replay(); episode(b_env, bufs[1]); same("replay %d" % k)
    episode(a_env, bufs[0]); episode(b_env, bufs[1]); same("eager episode 3 after replays")
    episode(a_env, bufs[0], ep=7); episode(b_env, bufs[1], ep=7); same("explicit episode 7")
    g.replay(); episode(b_env, bufs[1]); same("replay after an explicit episode: 8")
    a_env.close()
    b_env.close()

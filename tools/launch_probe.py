#!/usr/bin/env python3
"""Per-step wall time of the C2 bench loop under three launch paths (one process):
(a) ctypes launches, (b) ctypes launches + a HIP event pair per step, (c) one captured
HIP graph per episode (reset + 30 steps), replayed. Also checks (c) == (a) bit-exactly."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-for-im_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import C2_CONFIG  # noqa: E402
from imenv import VectorInvEnv  # noqa: E402
from imenv import _native as nat  # noqa: E402


def main(n=1 << 20, episodes=10):
    dev = torch.device("cuda:0")
    env = VectorInvEnv("MAIM", C2_CONFIG, n_envs=n, device=dev)
    T, N, F = env.T, env.N, env.F
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    actions = torch.rand((T, n, N), generator=g, device=dev) * 2 - 1
    obs_buf = torch.empty((T, n, N, F), device=dev)
    obs0 = torch.empty((n, N, F), device=dev)
    rew = torch.empty((T, n), dtype=torch.float64, device=dev)
    lib, h = env.lib, env._h

    def episode(sptr, events=None):
        nat.check(lib.imenv_reset(h, None, 0, 0, 0.0, None, -1, obs0.data_ptr(), 0, sptr), "reset")
        for t in range(T):
            if events is not None:
                events[t][0].record()
            nat.check(lib.imenv_step(h, actions[t].data_ptr(), 0, obs_buf[t].data_ptr(), 0, rew[t].data_ptr(),
                                     None, None, sptr), "step")
            if events is not None:
                events[t][1].record()

    sptr = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(2):
        episode(sptr)
    torch.cuda.synchronize()
    res = {}
    t0 = time.perf_counter()
    for _ in range(episodes):
        episode(sptr)
    torch.cuda.synchronize()
    res["a_ctypes"] = (time.perf_counter() - t0) / (episodes * T)
    evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(T)]
           for _ in range(episodes)]
    t0 = time.perf_counter()
    for k in range(episodes):
        episode(sptr, evs[k])
    torch.cuda.synchronize()
    res["b_ctypes_events"] = (time.perf_counter() - t0) / (episodes * T)
    kern = np.mean([a.elapsed_time(b) for ep in evs for a, b in ep]) * 1e-3
    # eager reference of two fresh episodes for the graph check
    nat.check(lib.imenv_reset(h, None, 0, 0, 0.0, None, 99, obs0.data_ptr(), 0, sptr), "reset")
    ref = []
    for t in range(T):
        nat.check(lib.imenv_step(h, actions[t].data_ptr(), 0, obs_buf[t].data_ptr(), 0, rew[t].data_ptr(),
                                 None, None, sptr), "step")
    ref.append((obs_buf[T - 1].clone(), rew.clone()))
    graph = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    cap.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.graph(graph, stream=cap):
        episode(torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    # replay with episode counter at 99 -> graph's auto reset makes it 100; eager ep 100 for comparison
    nat.check(lib.imenv_reset(h, None, 0, 0, 0.0, None, 99, obs0.data_ptr(), 0, sptr), "reset")
    torch.cuda.synchronize()
    graph.replay()
    torch.cuda.synchronize()
    got = (obs_buf[T - 1].clone(), rew.clone())
    nat.check(lib.imenv_reset(h, None, 0, 0, 0.0, None, 100, obs0.data_ptr(), 0, sptr), "reset")
    for t in range(T):
        nat.check(lib.imenv_step(h, actions[t].data_ptr(), 0, obs_buf[t].data_ptr(), 0, rew[t].data_ptr(),
                                 None, None, sptr), "step")
    torch.cuda.synchronize()
    assert torch.equal(got[0], obs_buf[T - 1]) and torch.equal(got[1], rew), "graph replay != eager"
    t0 = time.perf_counter()
    for _ in range(episodes):
        graph.replay()
    torch.cuda.synchronize()
    res["c_graph"] = (time.perf_counter() - t0) / (episodes * T)
    for k, v in res.items():
        print("%-18s %8.2f us/step  -> %.3e env-steps/s" % (k, v * 1e6, n / v))
    print("event-timed step kernel %.2f us" % (kern * 1e6))


if __name__ == "__main__":
    main()

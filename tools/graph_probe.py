#!/usr/bin/env python3
"""Per-step time of whole C2 episodes (reset + 30 steps), eager launches vs one HIP graph replay,
over env counts from launch-bound to bandwidth-bound. One JSON line per size."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "marl-for-im_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import C2_CONFIG  # noqa: E402


def main():
    from imenv import VectorInvEnv
    dev = torch.device("cuda", 0)
    sizes = [int(x) for x in sys.argv[1:]] or [4096, 16384, 65536, 131072, 262144, 1 << 20]
    for n in sizes:
        env = VectorInvEnv("MAIM", C2_CONFIG, n_envs=n, device=dev)
        T, N, F = env.T, env.N, env.F
        act = torch.rand((T, n, N), device=dev) * 2 - 1
        obs = torch.empty((T + 1, n, N, F), dtype=torch.float32, device=dev)
        rew = torch.empty((T, n), dtype=torch.float64, device=dev)

        def episode():
            env.reset(obs_out=obs[0])
            for t in range(T):
                env.step(act[t], obs_out=obs[t + 1], reward_out=rew[t])

        for _ in range(3):
            episode()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            episode()
        reps = 20
        res = {}
        for mode in ("eager", "graph", "eager", "graph"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(reps):
                if mode == "graph":
                    g.replay()
                else:
                    episode()
            e1.record()
            e1.synchronize()
            res[mode] = e0.elapsed_time(e1) * 1e3 / (reps * T)      # us per step, reset included
        print(json.dumps(dict(n_envs=n, eager_us_per_step=round(res["eager"], 3),
                              graph_us_per_step=round(res["graph"], 3),
                              eager_env_steps_per_s=round(n / res["eager"] * 1e6, 1),
                              graph_env_steps_per_s=round(n / res["graph"] * 1e6, 1))), flush=True)
        del g
        env.close()


if __name__ == "__main__":
    main()

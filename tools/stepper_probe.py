#!/usr/bin/env python3
"""Host cost of the step call: wall time per step of an eager rollout loop driven by
VectorInvEnv.step() (tensor checks per call) vs VectorInvEnv.rollout_stepper() (buffers validated
once), beside the kernel's own time, for a bench config at several batch sizes. Below the size
where the kernel outlasts the host call, the loop runs at the host's pace.

    python tools/stepper_probe.py [--config C2] [--sizes 65536,131072,262144,1048576] [--episodes 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "marl-for-im_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--sizes", default="65536,131072,262144,1048576")
    ap.add_argument("--episodes", type=int, default=10)
    args = ap.parse_args()
    import torch
    from bench import CONFIGS
    from imenv import VectorInvEnv
    dev = torch.device("cuda:0")
    kind, cfg = CONFIGS[args.config][:2]
    for n in (int(x) for x in args.sizes.split(",")):
        env = VectorInvEnv(kind, cfg, n_envs=n, device=dev)
        T, N, F = env.T, env.N, env.F
        acts = torch.rand((T, n, N), device=dev) * 2 - 1
        obs = torch.empty((T + 1, n, N, F), device=dev)
        rew = torch.empty((T,) + env.reward_shape(), dtype=torch.float64, device=dev)
        stepper = env.rollout_stepper(acts, obs, rew)

        def episode_step():
            env.reset(obs_out=obs[0])
            for t in range(T):
                env.step(acts[t], obs_out=obs[t + 1], reward_out=rew[t])

        def episode_stepper():
            env.reset(obs_out=obs[0])
            for t in range(T):
                stepper(t)

        out = dict(config=args.config, n_envs=n)
        for name, fn in (("step", episode_step), ("stepper", episode_stepper)):
            fn()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(args.episodes):
                fn()
            torch.cuda.synchronize(dev)
            out[name + "_us_per_step"] = round((time.perf_counter() - t0) / (args.episodes * T) * 1e6, 2)
        # kernel time alone: one episode's steps t = 1..T-1 between HIP events
        s = torch.cuda.current_stream(dev)
        env.reset(obs_out=obs[0])
        stepper(0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for t in range(1, T):
            stepper(t)
        e1.record(s)
        e1.synchronize()
        out["kernel_us"] = round(e0.elapsed_time(e1) * 1e3 / (T - 1), 2)
        out["stepper_env_steps_per_s"] = round(n / (out["stepper_us_per_step"] * 1e-6), 1)
        print(json.dumps(out), flush=True)
        env.close()


if __name__ == "__main__":
    main()

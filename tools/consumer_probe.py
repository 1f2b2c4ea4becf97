#!/usr/bin/env python3
"""Step kernel + the policy that consumes its observations, back to back on one stream: does a
store policy that speeds the step (non-temporal observation stores, set_store_policy("stream"))
cost the consumer that reads the observations right after? Times whole iterations of
    obs_t (written by step t-1) -> MLP policy (12 -> 64 -> 64 -> 4, float32, tanh) -> actions_t -> step t
on a bench config (C2 at 2^20 envs by default), plus the two parts alone (HIP events, 60 timed
iterations).

    python tools/consumer_probe.py [--config C2|C3|C4] [--n-envs 1048576] [--iters 60] [--store stream]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "marl-for-im_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-envs", type=int, default=1 << 20)
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--config", default="C2", help="bench.py config name (C2, C3, C4)")
    ap.add_argument("--store", default="default", choices=["default", "stream", "plain", "writethrough"])
    args = ap.parse_args()
    import torch
    from bench import CONFIGS
    from imenv import VectorInvEnv
    dev = torch.device("cuda:0")
    n, T = args.n_envs, 30
    kind, cfg = CONFIGS[args.config][:2]
    env = VectorInvEnv(kind, cfg, n_envs=n, device=dev)
    env.set_store_policy(args.store)
    N, F = env.N, env.F
    torch.manual_seed(0)
    policy = torch.nn.Sequential(torch.nn.Linear(N * F, 64), torch.nn.Tanh(), torch.nn.Linear(64, 64),
                                 torch.nn.Tanh(), torch.nn.Linear(64, N), torch.nn.Tanh()).to(dev)
    obs_buf = torch.empty((T + 1, n, N, F), dtype=torch.float32, device=dev)
    act_buf = torch.empty((T, n, N), dtype=torch.float32, device=dev)
    rew_buf = torch.empty((T,) + env.reward_shape(), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def iteration(s, do_policy=True, do_step=True):
        t = s % T
        if t == 0 and do_step:
            env.reset(obs_out=obs_buf[0])
        if do_policy:
            with torch.no_grad():
                torch.mul(policy(obs_buf[t].view(n, N * F)), 1.0, out=act_buf[t])
        if do_step:
            env.step(act_buf[t], obs_out=obs_buf[t + 1], reward_out=rew_buf[t])

    def timed(**kw):
        for s in range(2 * T):
            iteration(s, **kw)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for s in range(args.iters):
            iteration(s, **kw)
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / args.iters

    with torch.no_grad():
        act_buf.uniform_(-1, 1)
    both = timed()
    step_only = timed(do_policy=False)
    policy_only = timed(do_step=False)
    print(json.dumps(dict(config=args.config, n_envs=n, kernel=env.kernel_info(), us_per_iteration=round(both, 2),
                          us_step_alone=round(step_only, 2), us_policy_alone=round(policy_only, 2),
                          env_steps_per_s_with_policy=round(n / (both * 1e-6), 1),
                          store=args.store)))
    env.close()


if __name__ == "__main__":
    main()

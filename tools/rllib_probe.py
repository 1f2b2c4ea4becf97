#!/usr/bin/env python3
"""Throughput of the batched RLlib surfaces (imenv/rllib.py) as RLlib's sampler drives them: poll ->
actions for every (env, agent) -> send_actions, with try_reset per env at episode ends; a random
policy, so the number is the env side of a rollout worker (dict building included). Prints one JSON
line per (class, num_envs): env-steps/s and microseconds per batched step, beside the single-env
drop-in adaptor (the reference's per-env call shape).

    python tools/rllib_probe.py [--sizes 64,1024,16384] [--episodes 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-for-im_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", nargs="+", default=["64,1024,16384"])   # "64,1024" or "64 1024"
    ap.add_argument("--episodes", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import bench
    from imenv.envs import MultiAgentInvManagement
    from imenv.rllib import InvMultiAgentBaseEnv, InvVectorEnv
    cfg = bench.CONFIGS["C2"][1]
    rs = np.random.RandomState(0)
    for n in [int(x) for part in args.sizes for x in part.split(",") if x]:
        for cls, kind in ((InvMultiAgentBaseEnv, "MAIM"), (InvVectorEnv, "IM")):
            env = cls(kind, dict(cfg), num_envs=n)
            steps = 0
            t0 = None
            if cls is InvMultiAgentBaseEnv:
                ids = env.agent_ids
                obs = env.poll()[0]
                for ep in range(args.episodes + 1):
                    if ep == 1:
                        t0 = time.perf_counter()
                        steps = 0
                    for t in range(30):
                        a = rs.uniform(-1, 1, (n, len(ids)))
                        env.send_actions({i: {ag: a[i, k:k + 1] for k, ag in enumerate(ids)} for i in obs})
                        obs, rew, dones, infos, _ = env.poll()
                        steps += n
                    obs = {i: env.try_reset(i) for i in range(n)}
                env.stop()
            else:
                env.vector_reset()
                for ep in range(args.episodes + 1):
                    if ep == 1:
                        t0 = time.perf_counter()
                        steps = 0
                    for t in range(30):
                        env.vector_step(list(rs.uniform(-1, 1, (n, 4))))
                        steps += n
                    for i in range(n):
                        env.reset_at(i)
                env.close()
            el = time.perf_counter() - t0
            print(json.dumps({"surface": cls.__name__, "kind": kind, "num_envs": n,
                              "env_steps_per_s": round(steps / el, 1),
                              "us_per_batched_step": round(el / (steps / n) * 1e6, 1)}), flush=True)
    # the drop-in adaptor: one env per object, one kernel launch per env-step (the reference's shape)
    env = MultiAgentInvManagement(dict(cfg))
    ids = env.agent_names
    steps = 0
    for ep in range(args.episodes + 1):           # the first episode is untimed (kernel builds, first touch)
        if ep == 1:
            t0 = time.perf_counter()
            steps = 0
        env.reset()
        for t in range(30):
            env.step({ag: rs.uniform(-1, 1, 1) for ag in ids})
            steps += 1
    el = time.perf_counter() - t0
    print(json.dumps({"surface": "MultiAgentInvManagement (drop-in adaptor)", "num_envs": 1,
                      "env_steps_per_s": round(steps / el, 1), "us_per_step": round(el / steps * 1e6, 1)}), flush=True)
    env.close()


if __name__ == "__main__":
    main()

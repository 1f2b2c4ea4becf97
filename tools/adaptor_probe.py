#!/usr/bin/env python3
"""Host-side cost of the drop-in adaptors (one env, NumPy in / out, imenv/envs.py) per step(), next
to the oracle port of the reference step() on the same config: the latency a script that swaps the
class pays. One JSON line per class."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "marl-for-im_amd"), os.path.join(ROOT, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

from gen_fixtures import div1, serial4  # noqa: E402


def main():
    from imenv import envs
    cases = [("InvManagement", serial4(), lambda env, rs: rs.uniform(-1, 1, env.num_nodes)),
             ("MultiAgentInvManagement", dict(serial4(), independent=False),
              lambda env, rs: {k: rs.uniform(-1, 1, 1) for k in env.agent_names}),
             ("MultiAgentInvManagementDiv", dict(div1(), independent=False),
              lambda env, rs: {k: rs.uniform(-1, 1, 1) for k in env.agent_names})]
    for name, cfg, act in cases:
        env = getattr(envs, name)(dict(cfg))
        rs = np.random.RandomState(0)
        for _ in range(2):                      # warm: JIT compile, allocator
            env.reset()
            for _ in range(env.num_periods):
                env.step(act(env, rs))
        t_steps, t_resets, steps = 0.0, 0.0, 0
        for _ in range(10):
            t0 = time.perf_counter()
            env.reset()
            t1 = time.perf_counter()
            for _ in range(env.num_periods):
                env.step(act(env, rs))
            t2 = time.perf_counter()
            t_resets += t1 - t0
            t_steps += t2 - t1
            steps += env.num_periods
        print(json.dumps(dict(adaptor=name, us_per_step=round(t_steps / steps * 1e6, 1),
                              us_per_reset=round(t_resets / 10 * 1e6, 1))), flush=True)
        env.close()


if __name__ == "__main__":
    main()

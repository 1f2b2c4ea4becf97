#!/usr/bin/env python3
"""Does splitting a 2^20-env batch into G groups on G HIP streams hide the step kernel's ramp-up and
tail (each group's launch overlaps the other groups')? C2, whole episodes (reset + 30 steps), eager
launches, wall time per full step (all groups) with one synchronize at the end. One JSON line per G.

    python tools/stream_probe.py [total_envs]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "marl-for-im_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from bench import C2_CONFIG  # noqa: E402


def main():
    from imenv import VectorInvEnv
    dev = torch.device("cuda", 0)
    total = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    for G in (1, 2, 4, 8):
        n = total // G
        envs = [VectorInvEnv("MAIM", C2_CONFIG, n_envs=n, device=dev, env_offset=g * n) for g in range(G)]
        streams = [torch.cuda.Stream(dev) for _ in range(G)]
        T, N, F = envs[0].T, envs[0].N, envs[0].F
        act = torch.rand((T, total, N), device=dev) * 2 - 1
        obs = torch.empty((T + 1, total, N, F), dtype=torch.float32, device=dev)
        rew = torch.empty((T, total), dtype=torch.float64, device=dev)
        torch.cuda.synchronize()

        from imenv import _native as nat
        sp = [s.cuda_stream for s in streams]
        ptrs = [[(act[t, g * n:(g + 1) * n].data_ptr(), obs[t + 1, g * n:(g + 1) * n].data_ptr(),
                  rew[t, g * n:(g + 1) * n].data_ptr()) for g in range(G)] for t in range(T)]
        o0 = [obs[0, g * n:(g + 1) * n].data_ptr() for g in range(G)]
        lib = envs[0].lib
        hs = [e._h for e in envs]

        def episode():
            # raw C-ABI calls (as bench.py): the host cost per launch stays well under the kernel time
            for g in range(G):
                lib.imenv_reset(hs[g], None, nat.LAYOUT_DRAW, 0, 0.0, None, -1, o0[g], nat.F32, sp[g])
            for t in range(T):
                for g in range(G):
                    a, o, r = ptrs[t][g]
                    rc = lib.imenv_step(hs[g], a, nat.F32, o, nat.F32, r, None, None, sp[g])
                    if rc:
                        nat.check(rc, "imenv_step")

        for _ in range(3):
            episode()
        torch.cuda.synchronize()
        reps = 20
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            for _ in range(reps):
                episode()
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) * 1e6 / (reps * T)
            best = us if best is None else min(best, us)
        print(json.dumps(dict(groups=G, envs_per_group=n, us_per_step=round(best, 3),
                              env_steps_per_s=round(total / best * 1e6, 1))), flush=True)
        for e in envs:
            e.close()


if __name__ == "__main__":
    main()

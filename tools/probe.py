#!/usr/bin/env python3
"""Time the memory-pattern probes (tools/probe.hip) beside the real step kernel, interleaved
in one process (cdna_hip_programming.md §5.4 rule 24). Prints median us and GB/s per probe."""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "marl-for-im_amd"))
SRC = os.path.join(HERE, "probe.hip")
LIB = os.path.join(HERE, "_lib", "libprobe.so")


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                               "-o", LIB, SRC])


def main():
    build()
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        return
    import numpy as np
    import torch
    from bench import C2_CONFIG
    from imenv import VectorInvEnv
    from imenv import _native as nat
    n = 1 << 20
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(LIB)
    lib.probe_run.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_int64, ctypes.c_void_p]
    act = torch.rand((n, 4), device=dev)
    st = torch.zeros((16, n), dtype=torch.int32, device=dev)
    ring = torch.zeros((8, n, 4), dtype=torch.int32, device=dev)
    obs = torch.zeros((n, 12), dtype=torch.float32, device=dev)
    rew = torch.zeros(n, dtype=torch.float64, device=dev)
    src = torch.rand((5, n, 4), device=dev)
    dst = torch.zeros((8, n, 4), device=dev)
    env = VectorInvEnv("MAIM", C2_CONFIG, n_envs=n, device=dev)
    acts = torch.rand((30, n, 4), device=dev) * 2 - 1
    s = torch.cuda.current_stream(dev).cuda_stream
    obs_e = torch.empty((n, 4, 3), device=dev)
    rew_e = torch.empty(n, dtype=torch.float64, device=dev)
    env.reset()

    def run(which):
        if which < 3:
            a, b, c, d, e = ((act, st, ring, obs, rew) if which < 2 else (src, dst, None, None, None))
            ptr = lambda x: None if x is None else x.data_ptr()
            assert lib.probe_run(which, ptr(a), ptr(b), ptr(c), ptr(d), ptr(e), n, s) == 0
        else:
            if env.period >= 30:
                env.reset()
            env.step(acts[env.period], obs_out=obs_e, reward_out=rew_e)

    names = ["probe_soa", "probe_packed", "probe_copy", "imenv_step"]
    times = {k: [] for k in names}
    for w in range(2):
        for k in range(4):
            for _ in range(5):
                run(k)
    torch.cuda.synchronize()
    for rnd in range(40):
        for k in range(4):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            run(k)
            ev[1].record()
            ev[1].synchronize()
            times[names[k]].append(ev[0].elapsed_time(ev[1]) * 1e3)
    for k in names:
        us = float(np.median(times[k]))
        print("%-14s median %8.2f us  min %8.2f us  %7.1f GB/s (200 B/env)" % (k, us, min(times[k]),
                                                                           200 * n / us / 1e3))


if __name__ == "__main__":
    main()

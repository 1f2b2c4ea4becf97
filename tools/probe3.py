#!/usr/bin/env python3
"""Time the uint8-layout footprint probes (tools/probe3.hip) beside the real step kernel, interleaved
in one process; 29 back-to-back launches per HIP-event pair (as bench.py). Prints median us and
GB/s at 104 B/env (the C2 uint8 budget)."""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "marl-for-im_amd"))
SRC = os.path.join(HERE, "probe3.hip")
LIB = os.path.join(HERE, "_lib", "libprobe3.so")
NAMES = ["u8_bs256", "u8_bs512", "u8_ept2", "u8x4_bs64", "u8x4_bs128", "u8x4_bs256", "persist_g2048",
         "persist_g1024", "persist_g512"]


class P3Args(ctypes.Structure):
    _fields_ = [("act", ctypes.c_void_p), ("inv", ctypes.c_void_p), ("bl", ctypes.c_void_p),
                ("ou", ctypes.c_void_p), ("ring", ctypes.c_void_p), ("obs", ctypes.c_void_p),
                ("rew", ctypes.c_void_p), ("n", ctypes.c_int64), ("ring_row", ctypes.c_int32 * 4)]


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
    n = 1 << 20
    T = 30
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(LIB)
    lib.probe3_run.argtypes = [ctypes.c_int, ctypes.POINTER(P3Args), ctypes.c_void_p]
    act = torch.rand((T, n, 4), device=dev)
    st = torch.zeros((3, n), dtype=torch.int32, device=dev)
    ring = torch.zeros((7, n), dtype=torch.uint8, device=dev)
    obs = torch.zeros((T, n, 12), dtype=torch.float32, device=dev)
    rew = torch.zeros((T, n), dtype=torch.float64, device=dev)
    envs = []
    for ept in ("1", "2"):      # the JIT kernel is generated at the first step: pin EPT per env
        os.environ["IMENV_JIT_EPT"] = ept
        e = VectorInvEnv("MAIM", C2_CONFIG, n_envs=n, device=dev)
        e.reset()
        e.step(act[0], obs_out=obs[0].view(n, 4, 3), reward_out=rew[0])
        envs.append(e)
    s = torch.cuda.current_stream(dev).cuda_stream
    offs = [0, 1, 3, 6]
    delays = [1, 2, 3, 1]

    def args(t):
        a = P3Args(act[t].data_ptr(), st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr(), ring.data_ptr(),
                   obs[t].data_ptr(), rew[t].data_ptr(), n)
        for i in range(4):
            a.ring_row[i] = offs[i] + t % delays[i]
        return a

    pre = [args(t) for t in range(T)]

    def run_episode(which, evs):
        if which < len(NAMES):
            for t in range(T):
                if t == 1:
                    evs[0].record()
                assert lib.probe3_run(which, ctypes.byref(pre[t]), s) == 0
            evs[1].record()
        else:
            env = envs[which - len(NAMES)]
            env.reset()
            for t in range(T):
                if t == 1:
                    evs[0].record()
                env.step(act[t], obs_out=obs[t].view(n, 4, 3), reward_out=rew[t])
            evs[1].record()

    names = NAMES + ["imenv_step_ept1", "imenv_step_ept2"]
    times = {k: [] for k in names}
    for k in range(len(names)):
        run_episode(k, [torch.cuda.Event(enable_timing=True) for _ in range(2)])
    torch.cuda.synchronize()
    for rnd in range(8):
        for k in range(len(names)):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            run_episode(k, ev)
            ev[1].synchronize()
            times[names[k]].append(ev[0].elapsed_time(ev[1]) * 1e3 / (T - 1))
    for e in envs:
        print("step kernel:", e.kernel_info())
    for k in names:
        us = float(np.median(times[k]))
        print("%-14s median %8.2f us  min %8.2f us  %7.1f GB/s (104 B/env)" % (k, us, min(times[k]),
                                                                             104 * n / us / 1e3))


if __name__ == "__main__":
    main()

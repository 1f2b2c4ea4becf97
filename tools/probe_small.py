#!/usr/bin/env python3
"""Small-launch floors (tools/probe_small.hip) beside the real step kernel at the same env count,
interleaved in one process: an empty kernel of the step's grid, and the C2 step's exact loads and
stores (96 B per env-step) with plain or write-through stores and no arithmetic. 29 back-to-back
launches per HIP-event pair, 8 interleaved rounds; prints one JSON line of medians (us per launch)
and the HBM fraction of each at 96 B per env. Run it under rocprofv3 --kernel-trace --stats for the
trace's own per-kernel averages.

    python tools/probe_small.py [--n-envs 131072] [--rounds 8]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-for-im_amd")]
SRC = os.path.join(HERE, "probe_small.hip")
LIB = os.path.join(HERE, "bin", "libprobe_small.so")
NAMES = ["empty_bs64", "footprint_plain_bs64", "footprint_wt_bs64", "footprint_wt_bs256", "empty_bs256",
         "aos16_wt_bs64", "aos16_wt_bs256"]


class PSArgs(ctypes.Structure):
    _fields_ = [("act", ctypes.c_void_p), ("net", ctypes.c_void_p), ("ou", ctypes.c_void_p),
                ("ring", ctypes.c_void_p), ("obs", ctypes.c_void_p), ("rew", ctypes.c_void_p),
                ("n", ctypes.c_int64), ("ring_at", ctypes.c_int64 * 4)]


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                               "-o", LIB, SRC])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-envs", type=int, default=131072)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    build()
    if args.build_only:
        return
    import numpy as np
    import torch
    from bench import C2_CONFIG
    from imenv import VectorInvEnv
    from imenv import _native as nat
    n, T = args.n_envs, 30
    assert n % 256 == 0
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(LIB)
    lib.probe_small_run.argtypes = [ctypes.c_int, ctypes.POINTER(PSArgs), ctypes.c_void_p]
    act = torch.rand((T, n, 4), device=dev) * 2 - 1
    st = torch.zeros((4, n), dtype=torch.int32, device=dev)       # aos16 uses all 16 B per env of row 0..
    ring = torch.zeros((7, n), dtype=torch.uint8, device=dev)
    obs = torch.zeros((T, n, 4, 3), dtype=torch.float32, device=dev)
    rew = torch.zeros((T, n), dtype=torch.float64, device=dev)
    env = VectorInvEnv("MAIM", C2_CONFIG, n_envs=n, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    offs, delays = [0, 1, 3, 6], [1, 2, 3, 1]

    def pargs(t):
        a = PSArgs(act[t].data_ptr(), st[0].data_ptr(), st[1].data_ptr(), ring.data_ptr(), obs[t].data_ptr(),
                   rew[t].data_ptr(), n)
        for i in range(4):
            a.ring_at[i] = (offs[i] + t % delays[i]) * n
        return a

    pre = [pargs(t) for t in range(T)]
    h = env._h

    def episode(which, ev):
        if which < len(NAMES):
            for t in range(T):
                if t == 1:
                    ev[0].record()
                assert lib.probe_small_run(which, ctypes.byref(pre[t]), s) == 0
        else:
            nat.check(env.lib.imenv_reset(h, None, nat.LAYOUT_DRAW, 0, 0.0, None, -1, obs[0].data_ptr(), nat.F32, s),
                      "reset")
            for t in range(T):
                if t == 1:
                    ev[0].record()
                nat.check(env.lib.imenv_step(h, act[t].data_ptr(), nat.F32, obs[t].data_ptr(), nat.F32,
                                             rew[t].data_ptr(), None, None, s), "step")
        ev[1].record()

    names = NAMES + ["imenv_step"]
    times = {k: [] for k in names}
    for k in range(len(names)):          # warm: hipRTC build, first touch
        episode(k, [torch.cuda.Event(enable_timing=True) for _ in range(2)])
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for k in range(len(names)):
            torch.cuda._sleep(2000000)     # launches queue behind a busy-wait: the events time the GPU
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            episode(k, ev)
            ev[1].synchronize()
            times[names[k]].append(ev[0].elapsed_time(ev[1]) * 1e3 / (T - 1))
    out = {"n_envs": n, "kernel": env.kernel_info(), "bytes_per_env": 96, "us_per_launch": {}, "frac_96B": {},
           "note": "aos16_* move 104 B per env (16-byte state records); frac_96B prices every variant at 96 B"}
    for k in names:
        us = float(np.median(times[k]))
        out["us_per_launch"][k] = round(us, 3)
        out["frac_96B"][k] = round(96 * n / (us * 1e-6) / 8e12, 4)
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()

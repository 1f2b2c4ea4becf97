#!/usr/bin/env python3
"""Launch-cost probes (tools/probe_launch.hip) beside the production step kernel at one env count:
empty kernels with and without a by-value argument, the C2 step's bytes as 16-byte state records or as
the current rows, with pointers from a 384-byte by-value struct or as leading scalar arguments, each
from a plain build and from a build with kernel-argument preloading (-amdgpu-kernarg-preload-count=16).
29 back-to-back launches per HIP-event pair, queued behind a busy-wait, R interleaved rounds; one JSON
line of medians (us per launch). The kernel-argument placement is the HIP runtime's
(HIP_FORCE_DEV_KERNARG in the environment selects device memory): run the script once per setting.

    python tools/probe_launch.py [--n-envs 131072] [--rounds 8]
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
SRC = os.path.join(HERE, "probe_launch.hip")
LIBS = {"plain": (os.path.join(HERE, "bin", "libprobe_launch.so"), []),
        "preload": (os.path.join(HERE, "bin", "libprobe_launch_pre.so"),
                    ["-mllvm", "-amdgpu-kernarg-preload-count=16"])}
NAMES = ["empty_noarg", "empty_bigarg", "rec_bigarg", "rec_ptrs", "rows_ptrs", "rec_ptrs_bs128", "rec_ptrs_bs256"]


class PLArgs(ctypes.Structure):
    _fields_ = [("act", ctypes.c_void_p), ("rec", ctypes.c_void_p), ("net", ctypes.c_void_p), ("ou", ctypes.c_void_p),
                ("ring", ctypes.c_void_p * 4), ("obs", ctypes.c_void_p), ("rew", ctypes.c_void_p), ("n", ctypes.c_int64)]


def build():
    os.makedirs(os.path.join(HERE, "bin"), exist_ok=True)
    for lib, extra in LIBS.values():
        if not os.path.exists(lib) or os.path.getmtime(lib) < os.path.getmtime(SRC):
            subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared"] + extra +
                                  ["-o", lib, SRC])


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
    libs = {}
    for k, (path, _) in LIBS.items():
        libs[k] = ctypes.CDLL(path)
        libs[k].probe_launch_run.argtypes = [ctypes.c_int, ctypes.POINTER(PLArgs), ctypes.c_void_p]
    act = torch.rand((T, n, 4), device=dev) * 2 - 1
    rec = torch.zeros((n, 4), dtype=torch.int32, device=dev)
    rows = torch.zeros((2, n), dtype=torch.int32, device=dev)
    ring = torch.zeros((7, n), dtype=torch.uint8, device=dev)
    obs = torch.zeros((T, n, 4, 3), dtype=torch.float32, device=dev)
    rew = torch.zeros((T, n), dtype=torch.float64, device=dev)
    env = VectorInvEnv("MAIM", C2_CONFIG, n_envs=n, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    offs, delays = [0, 1, 3, 6], [1, 2, 3, 1]

    def pargs(t):
        a = PLArgs()
        a.act, a.rec, a.net, a.ou = act[t].data_ptr(), rec.data_ptr(), rows[0].data_ptr(), rows[1].data_ptr()
        for i in range(4):
            a.ring[i] = ring.data_ptr() + (offs[i] + t % delays[i]) * n
        a.obs, a.rew, a.n = obs[t].data_ptr(), rew[t].data_ptr(), n
        return a

    pre = [pargs(t) for t in range(T)]
    h = env._h
    variants = [(b, k, nm) for b in LIBS for k, nm in enumerate(NAMES)] + [("prod", -1, "imenv_step")]

    def episode(v, ev):
        b, k, _ = v
        if b != "prod":
            for t in range(T):
                if t == 1:
                    ev[0].record()
                assert libs[b].probe_launch_run(k, ctypes.byref(pre[t]), s) == 0
        else:
            nat.check(env.lib.imenv_reset(h, None, nat.LAYOUT_DRAW, 0, 0.0, None, -1, obs[0].data_ptr(), nat.F32, s),
                      "reset")
            for t in range(T):
                if t == 1:
                    ev[0].record()
                nat.check(env.lib.imenv_step(h, act[t].data_ptr(), nat.F32, obs[t].data_ptr(), nat.F32,
                                             rew[t].data_ptr(), None, None, s), "step")
        ev[1].record()

    key = lambda v: v[2] if v[0] == "prod" else "%s:%s" % (v[0], v[2])
    times = {key(v): [] for v in variants}
    for v in variants:            # warm: hipRTC build, first touch
        episode(v, [torch.cuda.Event(enable_timing=True) for _ in range(2)])
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for v in variants:
            torch.cuda._sleep(2000000)     # launches queue behind a busy-wait: the events time the GPU
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            episode(v, ev)
            ev[1].synchronize()
            times[key(v)].append(ev[0].elapsed_time(ev[1]) * 1e3 / (T - 1))
    out = {"n_envs": n, "kernel": env.kernel_info(), "HIP_FORCE_DEV_KERNARG": os.environ.get("HIP_FORCE_DEV_KERNARG"),
           "us_per_launch": {}, "us_min": {},
           "note": "rec_* move 104 B per env (16-byte records); rows_* and imenv_step 96 B"}
    for k, v in times.items():
        out["us_per_launch"][k] = round(float(np.median(v)), 3)
        out["us_min"][k] = round(float(np.min(v)), 3)
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()

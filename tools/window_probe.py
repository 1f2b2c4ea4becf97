#!/usr/bin/env python3
"""Where the driver's short timed window goes at small launches (C2 at 131,072 envs: C5's per-GPU shard;
the driver's --steps 20 --warmup 5). Replays bench.py's window (barrier-free: one process) R times per
variant with a HIP event after every launch, and reports per variant: the wall time of the window, the
GPU time from the first launch's start to the last launch's end, the host's enqueue time, and the
per-launch durations by position (median over the R windows).

Variants: "plain" (bench.py's window as it is), "lead50" (a 50 us busy-wait lead), "burn" (a 40 us ALU
kernel in front of the window, outside the timing: is the first launch of a window slow because the
clocks dropped while the GPU idled?), "burn_in" (the same kernel inside the window); with --no-events
(no event after each launch: the host enqueues at its real pace, wall and GPU-span only) also
"spinsync" (the window's end waits by polling an event instead of a blocking synchronize).

    python tools/window_probe.py [--n-envs 131072] [--steps 20] [--rounds 15]
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
    ap.add_argument("--n-envs", type=int, default=131072)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--no-events", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from imenv import VectorInvEnv
    from imenv import _native as nat
    n, K, W = a.n_envs, a.steps, a.warmup
    dev = torch.device("cuda:0")
    env = VectorInvEnv("MAIM", bench.C2_CONFIG, n_envs=n, device=dev)
    T = env.T
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    act = torch.rand((T, n, 4), generator=g, device=dev) * 2 - 1
    obs = torch.empty((T, n, 4, 3), device=dev)
    rew = torch.empty((T, n), dtype=torch.float64, device=dev)
    obs0 = torch.empty((n, 4, 3), device=dev)
    lib, h = env.lib, env._h
    st = torch.cuda.current_stream(dev)
    sp = st.cuda_stream
    phase = bench.episode_phase(W, K, T)
    burn_x = torch.ones(1 << 16, device=dev)

    def burn():            # ~40 us of dependent ALU work on the whole chip (raises the clocks)
        y = burn_x
        for _ in range(20):
            y = torch.sin(y) * 1.0001
        return y

    def steps(first, cnt, evs=None):
        for s in range(first, first + cnt):
            t = (s + phase) % T
            if t == 0:
                nat.check(lib.imenv_reset(h, None, nat.LAYOUT_DRAW, 0, 0.0, None, -1, obs0.data_ptr(), nat.F32, sp),
                          "reset")
            nat.check(lib.imenv_step(h, act[t].data_ptr(), nat.F32, obs[t].data_ptr(), nat.F32, rew[t].data_ptr(),
                                     None, None, sp), "step")
            if evs is not None:
                evs.append(torch.cuda.Event(enable_timing=True))
                evs[-1].record(st)

    us_per_cycle = None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    torch.cuda._sleep(200000)
    e1.record(st)
    e1.synchronize()
    us_per_cycle = e0.elapsed_time(e1) * 1e3 / 200000
    out = {"n_envs": n, "steps": K, "warmup": W, "phase": phase, "variants": {}}
    variants = ("plain", "lead50", "burn", "burn_in") + (("spinsync", "lead50_spinsync") if a.no_events else ())
    for var in variants:
        walls, gpus, hosts, per = [], [], [], []
        for r in range(a.rounds + 1):
            steps(-phase, phase + W)              # reset + positioning + warmup, as bench.warm()
            if var == "burn":
                burn()
            torch.cuda.synchronize(dev)
            start = torch.cuda.Event(enable_timing=True)
            evs = []
            t0 = time.perf_counter()
            if var == "burn_in":
                burn()
            if var.startswith("lead50"):
                torch.cuda._sleep(int(50 / us_per_cycle))
            start.record(st)
            steps(W, K, None if a.no_events else evs)
            if a.no_events:
                evs.append(torch.cuda.Event(enable_timing=True))
                evs[-1].record(st)
            th = time.perf_counter()
            if var.endswith("spinsync"):
                while not evs[-1].query():
                    pass
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            if r == 0:
                continue                           # the first window of a variant builds / warms
            walls.append((t1 - t0) * 1e6)
            hosts.append((th - t0) * 1e6)
            gpus.append(start.elapsed_time(evs[-1]) * 1e3)
            prev = start
            d = []
            for e in evs:
                d.append(prev.elapsed_time(e) * 1e3)
                prev = e
            per.append(d)
        per = np.median(np.array(per), axis=0)
        out["variants"][var] = {"wall_us": round(float(np.median(walls)), 1),
                                "gpu_first_to_last_us": round(float(np.median(gpus)), 1),
                                "host_enqueue_us": round(float(np.median(hosts)), 1),
                                "per_launch_us_by_position": [round(float(x), 2) for x in per]}
        print(json.dumps({var: out["variants"][var]}), flush=True)
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()

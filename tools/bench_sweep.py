#!/usr/bin/env python3
"""Step-kernel roofline over every golden configuration (tests/golden: all four env classes and the
observation-flag combinations the reference's scripts use), not only the bench workload.

    python tools/bench_sweep.py [--n-envs 1048576] [--out gpurun_out/sweep.jsonl] [--obs-f64] [--store stream]
                                [--fuzz]

Per config: float32 actions, float32 observations (--obs-f64: float64), in-kernel Philox demand (and noisy delay where the case
has it), 2 warmup + 2 timed episodes; the step kernel is timed with HIP events on its stream over
launches t = 1..T-1 of each timed episode, queued behind a GPU busy-wait so that small launches are
timed back to back rather than at the host's pace (round 3). achieved = VectorInvEnv.step_traffic() bytes x n / time.
One JSON line per config.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "marl-for-im_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from golden_io import case_names, fuzz_case_names, load_case  # noqa: E402

HBM_PEAK_GBS = 8000.0


_CYCLES_PER_US = {}


def spin_cycles(dev, us):
    """torch.cuda._sleep cycles for about `us` microseconds (calibrated once per device with events)."""
    if dev not in _CYCLES_PER_US:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        torch.cuda._sleep(200000)
        e1.record()
        e1.synchronize()
        _CYCLES_PER_US[dev] = 200000 / (e0.elapsed_time(e1) * 1e3)
    return int(us * _CYCLES_PER_US[dev])


def run_case(name, n, dev, obs_dtype=torch.float32, store="default"):
    from imenv import VectorInvEnv
    meta, _ = load_case(name)
    env = VectorInvEnv(meta["kind"], meta["config"], n_envs=n, device=dev)
    env.set_store_policy(store)
    N, T = env.N, env.T
    noisy = float(meta["noisy"])
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    acts = torch.rand((T, n, N), generator=g, device=dev) * 2 - 1
    obs = torch.empty((n, N, env.F), dtype=obs_dtype, device=dev)
    rew = torch.empty(env.reward_shape(), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    times = []
    for ep in range(4):
        env.reset(noisy_delay=noisy > 0, noisy_delay_threshold=noisy, obs_out=obs)
        e0 = e1 = None
        for t in range(T):
            if t == 1 and ep >= 2:
                # a GPU busy-wait longer than the host's enqueue of the episode's remaining steps: the
                # timed launches queue up behind it and run back to back (eager step() costs ~6-8 us of
                # host time, more than a small launch's kernel)
                torch.cuda._sleep(spin_cycles(dev, (T - 1) * 20.0))
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            env.step(acts[t], obs_out=obs, reward_out=rew)
        if e0 is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(stream)
            e1.synchronize()
            times.append(e0.elapsed_time(e1) / (T - 1))
    us = float(np.mean(times)) * 1e3
    steady, avg = env.step_traffic(obs_bytes=obs.element_size())
    gbs = avg * n / (us * 1e-6) / 1e9
    out = dict(case=name, kind=meta["kind"], N=N, F=env.F, obs=str(obs_dtype).split(".")[-1], state_bytes=env.state_layout()[0],
               reward=("independent" if env.spec.reward_mode == 2 else "scalar"), noisy_delay=noisy,
               n_envs=n, kernel_us=round(us, 3), env_steps_per_s=round(n / (us * 1e-6), 1),
               bytes_per_env_step=round(avg, 3), achieved_gbs=round(gbs, 1), frac=round(gbs / HBM_PEAK_GBS, 4),
               store_policy=store, kernel=env.kernel_info())
    env.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-envs", type=int, default=1 << 20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--cases", default=None, help="comma-separated subset")
    ap.add_argument("--obs-f64", action="store_true", help="float64 observations (the reference's dtype)")
    ap.add_argument("--store", default="default", choices=["default", "stream"], help="step-kernel store policy")
    ap.add_argument("--fuzz", action="store_true", help="also the drawn configurations of tests/golden/fuzz")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    names = args.cases.split(",") if args.cases else case_names() + (fuzz_case_names() if args.fuzz else [])
    fo = open(args.out, "w") if args.out else None
    for name in names:
        r = run_case(name, args.n_envs, dev, torch.float64 if args.obs_f64 else torch.float32, args.store)
        line = json.dumps(r)
        print(line, flush=True)
        if fo:
            fo.write(line + "\n")
            fo.flush()


if __name__ == "__main__":
    main()

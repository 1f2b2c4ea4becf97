#!/usr/bin/env python3
"""Throughput of the fused plan replay (imenv_plan_rollout): the LP scripts' evaluation loop.

    python tools/bench_plan.py [--config SHLP8|SHLP4|SHLP_div1] [--plans P] [--scenarios S]
                               [--layout episode|shared] [--f32] [--no-rewards] [--reps K] [--no-cpu]

Workload (default): SHLP_8.py's replay (InvManagement 8-stage, SHLP_8.py:26-46 constants,
standardise_state / standardise_actions False as its DFO_CONFIG), one plan per demand scenario
(the per-scenario LP of SHLP_8.py:737-766) as float64 actions [T][S][N], the scenarios' customer
demand as a host-drawn Poisson(5) table [T][R][S], per-step rewards (profit[j, t]) and per-episode
metrics written out. One unit of work = one env-step; value = P * S * T / launch time (HIP events on
the launch's stream, K launches).

Roofline: HBM. Algorithmic bytes per env-step = plan row (8N f64 / 4N f32; 0 for a shared plan, a
broadcast read) + demand (4R) + reward (8, optional) + the per-episode metrics (5 x 8 B / T). The
arithmetic (the step's ~300-600 VALU instructions per env-step) runs under it; bench_rollout.py's VALU
numbers bound the shared-plan form. The CPU baseline is the oracle port of the scripts' loop
(oracle/plan.py over one env, one scenario per call) on this host's cores.
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "marl-for-im_amd"), os.path.join(ROOT, "tools")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

from gen_fixtures import div1, serial4, serial8  # noqa: E402

HBM_PEAK_GBS = 8000.0
RAW = dict(standardise_state=False, standardise_actions=False)
CONFIGS = {
    "SHLP8": ("IM", serial8(**RAW)),
    "SHLP4": ("IM", serial4(**RAW)),
    "SHLP_div1": ("IM_div", div1(**RAW)),
}


def _cpu_worker(args):
    name, seconds, seed = args
    from oracle import plan as pl
    kind, cfg = CONFIGS[name]
    rs = np.random.RandomState(seed)
    N = cfg.get("num_stages", cfg.get("num_nodes"))
    R = 1 if kind == "IM" else 2
    steps, t0 = 0, time.perf_counter()
    while True:
        dem = rs.poisson(5, size=(1, R, 30))
        plan = rs.randint(0, 20, size=(30, 1, 1, N)).astype(np.float64)
        pl.plan_rollout(kind, cfg, plan, per_episode=True, demand=dem[:, 0] if R == 1 else dem)
        steps += 30
        el = time.perf_counter() - t0
        if el >= seconds:
            return steps, el


def cpu_baseline(name, seconds):
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    with mp.get_context("fork").Pool(cores) as pool:
        res = pool.map(_cpu_worker, [(name, seconds, 100 + i) for i in range(cores)])
    total = sum(s / e for s, e in res)
    return dict(value=round(total, 1), unit="env-steps/s", cores=cores, kind="port",
                sample="oracle/plan.py replay loop, 1 scenario per call, %d processes x %.1f s" % (cores, seconds))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="SHLP8", choices=sorted(CONFIGS))
    ap.add_argument("--plans", type=int, default=1)
    ap.add_argument("--scenarios", type=int, default=1 << 20)
    ap.add_argument("--layout", default="episode", choices=["episode", "shared"])
    ap.add_argument("--f32", action="store_true", help="float32 plans (default float64, the LP's values)")
    ap.add_argument("--drawn", action="store_true", help="in-kernel Philox demand instead of a host table")
    ap.add_argument("--no-rewards", action="store_true")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=1.0)
    args = ap.parse_args()
    kind, cfg = CONFIGS[args.config]
    cpu = None if args.no_cpu else cpu_baseline(args.config, args.cpu_seconds)   # before the GPU

    import torch
    from imenv.plan import PlanRollout
    dev = torch.device("cuda", 0)
    pr = PlanRollout(kind, cfg, device=dev)
    P, S, T, N, R = args.plans, args.scenarios, pr.T, pr.N, pr.R
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    dt = torch.float32 if args.f32 else torch.float64
    per_ep = args.layout == "episode"
    shape = (P, S, T, N) if per_ep else (P, T, N)
    plans = torch.randint(0, 20, shape, generator=g, device=dev).to(dt)
    demand = None if args.drawn else torch.poisson(torch.full((S, R, T), 5.0, device=dev), generator=g).to(torch.int32)
    if demand is not None and kind == "IM":
        demand = demand[:, 0]
    # the kernel's layouts, prepared once outside the timed region (run() would permute per call)
    x, _, _ = pr._plans(plans, per_ep, S)
    table = pr._ro._demand_table(demand) if demand is not None else None
    del plans, demand
    rw = not args.no_rewards

    def launch(ep):
        from ctypes import byref, c_void_p
        from imenv import _native as nat
        a = nat.ImEnvPlanRollout()
        a.actions = x.data_ptr()
        a.action_dtype = nat.F64 if x.dtype == torch.float64 else nat.F32
        a.plan_layout = nat.PLAN_PER_EPISODE if per_ep else nat.PLAN_SHARED
        a.num_plans, a.num_scenarios = P, S
        a.demand = table.data_ptr() if table is not None else None
        a.episode = ep
        a.rewards = rew.data_ptr() if rw else None
        a.episode_stats = eps.data_ptr()
        a.policy_stats = stats.data_ptr()
        nat.check(pr._env.lib.imenv_plan_rollout(pr._env._h, byref(a), c_void_p(stream.cuda_stream)),
                  "imenv_plan_rollout")

    rew = torch.empty((T, P, S), dtype=torch.float64, device=dev)
    eps = torch.empty((5, P, S), dtype=torch.float64, device=dev)
    stats = torch.empty((P, 5, 2), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    for k in range(2):
        launch(k)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
    t0 = time.perf_counter()
    for k in range(args.reps):
        ev[k][0].record(stream)
        launch(k + 2)
        ev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    steps = P * S * T
    esz = 8 if dt == torch.float64 else 4
    b_step = (esz * N if per_ep else 0) + (4 * R if table is not None else 0) + (8 if rw else 0) + 40.0 / T
    ach = steps * b_step / (ms * 1e-3) / 1e9
    res = {
        "metric": "plan replay env-steps/s (P plans x S scenarios x T periods per launch)",
        "value": round(steps / (ms * 1e-3), 1),
        "unit": "env-steps/s",
        "ms_per_launch": round(ms, 4),
        "wall_env_steps_per_s": round(steps * args.reps / wall, 1),
        "config": {"workload": "%s LP replay (raw state/actions), %s plans (%s), %s demand" %
                               (args.config, args.layout, "f32" if args.f32 else "f64",
                                "in-kernel Poisson(5)" if table is None else "host Poisson(5) table"),
                   "plans": P, "scenarios": S, "num_periods": T, "rewards_out": rw},
        "kernel": pr.kernel_info(),
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4), "bytes_per_env_step": round(b_step, 3)},
        "mean_return_plan0": float(stats[0, 0, 0].item()),
        "cpu_baseline": cpu,
    }
    if cpu:
        res["gpu_over_cpu"] = round(res["value"] / cpu["value"], 1)
    print(json.dumps(res), flush=True)
    pr.close()


if __name__ == "__main__":
    main()

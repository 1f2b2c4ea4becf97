#!/usr/bin/env python3
"""Throughput of the fused base-stock rollout (imenv_base_stock_rollout), §8f row 1.

    python tools/bench_rollout.py [--policies P] [--scenarios S] [--reps K] [--kind IM] [--no-cpu]

Workload: the reference's DFO setting (inv_management.py:119-130: InvManagement 4-stage,
inv_management.py:35-56 constants, unstandardised state/actions), P candidate order-up-to policies
x S in-kernel Poisson(5) demand scenarios per launch, dfo_func objective on. A unit of work is one
env-step (one period of one episode); value = P * S * T / launch time (HIP events on the launch's
stream, K launches). The kernel is compute-bound (no per-step HBM traffic: state in registers,
queue in LDS), so its roofline is VALU issue: SQ_INSTS_VALU (PMC, tools/profile_rollout.sh) over
the launch time against 256 CUs x 4 SIMDs x 0.5 wave-instructions/cycle x 2.4 GHz.
The CPU baseline is the oracle port of dfo_func (oracle/base_stock.py over one env, as the
reference runs it) on this host's cores.
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

VALU_PEAK = 256 * 4 * 0.5 * 2.4e9      # wave-instructions / s (MI355X_MICROARCH.md: SIMD issues a wave64 VALU op / 2 cyc)
CONFIGS = {
    "IM": ("IM", serial4(standardise_state=False, standardise_actions=False)),
    "IM8": ("IM", serial8(standardise_state=False, standardise_actions=False)),
    "IM_div1": ("IM_div", div1(standardise_state=False, standardise_actions=False)),
}


def _cpu_worker(args):
    kind, name, seconds, seed = args
    from scipy.stats import poisson
    from oracle import base_stock as bs
    cfg = CONFIGS[name][1]
    rs = np.random.RandomState(seed)
    N = cfg.get("num_stages", cfg.get("num_nodes"))
    pmf = lambda k: poisson.pmf(k, mu=5)  # noqa: E731
    steps, t0 = 0, time.perf_counter()
    while True:
        R = 1 if kind == "IM" else 2
        dem = rs.poisson(5, size=(1, R, 30))
        bs.rollout(kind, cfg, rs.uniform(0, 40, size=(1, N)), demand=dem[:, 0] if R == 1 else dem, pmf=pmf)
        steps += 30
        el = time.perf_counter() - t0
        if el >= seconds:
            return steps, el


def cpu_baseline(kind, name, seconds):
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    with mp.get_context("fork").Pool(cores) as pool:
        res = pool.map(_cpu_worker, [(kind, name, seconds, 100 + i) for i in range(cores)])
    total = sum(s / e for s, e in res)
    return dict(value=round(total, 1), unit="env-steps/s", cores=cores, kind="port",
                sample="oracle/base_stock.py dfo_func restatement, 1 episode per call, %d processes x %.1f s"
                       % (cores, seconds))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="IM", choices=sorted(CONFIGS))
    ap.add_argument("--policies", type=int, default=64)
    ap.add_argument("--scenarios", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-objective", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=1.0)
    args = ap.parse_args()
    kind, cfg = CONFIGS[args.config]
    cpu = None if args.no_cpu else cpu_baseline(kind, args.config, args.cpu_seconds)   # before the GPU

    import torch
    from imenv.policy import BaseStockRollout
    dev = torch.device("cuda", 0)
    ro = BaseStockRollout(kind, cfg, device=dev)
    P, S, T = args.policies, args.scenarios, ro.T
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    pol = torch.rand((P, ro.N), generator=g, device=dev, dtype=torch.float64) * 40
    stream = torch.cuda.current_stream(dev)
    obj = not args.no_objective
    assert torch.isfinite(pol).all()     # validated once: the timed launches skip run()'s per-call check (a sync)
    for _ in range(2):
        ro.run(pol, n_scenarios=S, episode=0, objective=obj, per_episode=True, check_finite=False)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
    t0 = time.perf_counter()
    for k in range(args.reps):
        ev[k][0].record(stream)
        out = ro.run(pol, n_scenarios=S, episode=k + 1, objective=obj, per_episode=True, check_finite=False)
        ev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    steps = P * S * T
    res = {
        "metric": "base-stock rollout env-steps/s (P policies x S scenarios x T periods per launch)",
        "value": round(steps / (ms * 1e-3), 1),
        "unit": "env-steps/s",
        "ms_per_launch": round(ms, 4),
        "wall_env_steps_per_s": round(steps * args.reps / wall, 1),
        "config": {"workload": args.config + " DFO config (unstandardised), in-kernel Poisson(5) demand",
                   "policies": P, "scenarios": S, "num_periods": T, "objective": obj},
        "kernel": ro.kernel_info(),
        "valu_peak_wave_instr_per_s": VALU_PEAK,
        "mean_objective_policy0": float(out["stats"][0, 1, 0].item()),
        "cpu_baseline": cpu,
    }
    # VALU-issue roofline from the committed PMC summary of this exact kernel variant
    # (tools/profile_rollout.sh -> profiles/pmc_rollout_kernel.json): SQ_INSTS_VALU per launch over the
    # rocprof-measured average duration of the rollout kernel alone
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_rollout_kernel.json")) as f:
            pmc = json.load(f)
        if pmc.get("kernel_info") and pmc["kernel_info"] in ro.kernel_info() and pmc.get("policies") == P \
                and pmc.get("scenarios") == S:
            ach = pmc["valu_wave_instr_per_launch"] / (pmc["kernel_avg_ns"] * 1e-9)
            res["roofline"] = {"bound": "valu", "achieved": round(ach, 1), "peak": VALU_PEAK, "unit": "wave-instr/s",
                               "frac": round(ach / VALU_PEAK, 4),
                               "valu_instr_per_env_step": round(pmc["valu_wave_instr_per_launch"] * 64 / steps, 1),
                               "source": "profiles/pmc_rollout_kernel.json"}
            if pmc.get("issue_model"):   # per-class issue costs (tools/probe_valu.hip): [low, high]
                res["roofline"]["issue_model_frac"] = pmc["issue_model"]["frac"]
    except (OSError, ValueError, KeyError):
        pass
    if cpu:
        res["gpu_over_cpu"] = round(res["value"] / cpu["value"], 1)
    print(json.dumps(res), flush=True)
    ro.close()


if __name__ == "__main__":
    main()

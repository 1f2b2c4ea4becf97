#!/usr/bin/env python3
"""Per-wave phase timeline of one step-kernel launch (diagnostic kernel build with -DIMENV_STAMPS=1:
s_memrealtime stamps at entry, loads issued, loads landed (an added vmcnt(0) wait), computed, slab
barrier, stores issued, stores acknowledged). Prints the distribution of each phase over the waves and
the launch's span, in microseconds (100 MHz counter).

    IMENV_DIAG=1 IMENV_STAMPS=1 IMENV_JIT_OPTS=-DIMENV_STAMPS=1 python tools/stamp_probe.py --config C4 [--n-envs N] [--store S]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "marl-for-im_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

PHASES = ["issue_loads", "wait_loads", "compute", "barrier", "issue_stores", "drain_stores"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--n-envs", type=int, default=None)
    ap.add_argument("--store", default="default")
    ap.add_argument("--steps", type=int, default=40)
    args = ap.parse_args()
    assert os.environ.get("IMENV_STAMPS") == "1" and "IMENV_STAMPS" in os.environ.get("IMENV_JIT_OPTS", "")
    assert os.environ.get("IMENV_DIAG") == "1", "a diagnostic kernel build needs IMENV_DIAG=1 (imenv_jit.hip)"
    import numpy as np
    import torch
    from bench import CONFIGS
    from imenv import VectorInvEnv
    kind, cfg, _, nd = CONFIGS[args.config]
    n = args.n_envs or nd
    dev = torch.device("cuda:0")
    env = VectorInvEnv(kind, cfg, n_envs=n, device=dev)
    env.set_store_policy(args.store)
    T, N, F = env.T, env.N, env.F
    act = torch.rand((T, n, N), device=dev) * 2 - 1
    obs = torch.empty((T + 1, n, N, F), device=dev)
    rew = torch.empty((T,) + env.reward_shape(), dtype=torch.float64, device=dev)
    rows = []
    for s in range(args.steps):
        t = s % T
        if t == 0:
            env.reset(obs_out=obs[0])
        env.step(act[t], obs_out=obs[t + 1], reward_out=rew[t])
        if s >= T and t in (5, 15, 25):      # second episode on: warm, mid-episode periods
            cnt = ctypes.c_int64()
            env.lib.imenv_debug_stamps(env._h, None, 0, ctypes.byref(cnt))
            buf = np.zeros(cnt.value, dtype=np.uint64)
            env.lib.imenv_debug_stamps(env._h, buf.ctypes.data, cnt.value, ctypes.byref(cnt))
            st = buf.reshape(-1, 8)
            st = st[st[:, 0] > 0].astype(np.int64)
            rows.append(st)
    out = {"config": args.config, "n_envs": n, "kernel": env.kernel_info(), "store": args.store, "launches": []}
    assert out["kernel"].startswith("jit-diag:"), out["kernel"]     # the stamps build, not an AOT fallback
    for st in rows:
        t0 = st[:, 0].min()
        d = np.diff(st[:, :7], axis=1) / 100.0       # 10 ns ticks -> us
        rec = {"waves": int(st.shape[0]), "span_us": round((st[:, 6].max() - t0) / 100.0, 3),
               "first_end_us": round((st[:, 6].min() - t0) / 100.0, 3),
               "last_start_us": round((st[:, 0].max() - t0) / 100.0, 3)}
        for k, ph in enumerate(PHASES):
            rec[ph] = [round(float(np.percentile(d[:, k], q)), 3) for q in (10, 50, 90)]
        for k in range(7):
            rec["t%d_p50_us" % k] = round(float(np.percentile(st[:, k] - t0, 50)) / 100.0, 3)
        xcc = (st[:, 7] >> 32) & 0xF
        rec["span_by_xcc_us"] = [round(float((st[xcc == x, 6].max() - st[xcc == x, 0].min()) / 100.0), 3)
                                 for x in range(8) if (xcc == x).any()]
        out["launches"].append(rec)
    print(json.dumps(out))
    env.close()


if __name__ == "__main__":
    main()

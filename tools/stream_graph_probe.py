#!/usr/bin/env python3
"""Can independent env groups on separate HIP streams hide each other's launch boundary at C5's
per-GPU size? C2 at `total` envs (default 131,072) split into G handles (env ids contiguous), each
stepped on its own stream, one episode (reset + 30 steps) per group:

  eager   launches queued behind a GPU busy-wait (the host enqueues every group's episode first, so
          the events time the GPU, not the host's pace)
  graph   the G episodes captured into ONE HIP graph (fork / join over the G streams) and replayed

Prints one JSON line per (mode, G): GPU microseconds per full step (all groups, reset included) and
the env-steps/s that gives. Same kernels, same results as one handle (the envs are independent).

    python tools/stream_graph_probe.py [--total 131072] [--groups 1,2,4] [--reps 10]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-for-im_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total", type=int, default=131072)
    ap.add_argument("--groups", default="1,2,4")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch
    from bench import C2_CONFIG
    from imenv import VectorInvEnv
    from imenv import _native as nat
    dev = torch.device("cuda", 0)
    total = args.total
    for G in [int(x) for x in args.groups.split(",")]:
        n = total // G
        envs = [VectorInvEnv("MAIM", C2_CONFIG, n_envs=n, device=dev, env_offset=g * n) for g in range(G)]
        streams = [torch.cuda.Stream(dev) for _ in range(G)]
        T, N, F = envs[0].T, envs[0].N, envs[0].F
        act = torch.rand((T, total, N), device=dev) * 2 - 1
        obs = torch.empty((T + 1, total, N, F), dtype=torch.float32, device=dev)
        rew = torch.empty((T, total), dtype=torch.float64, device=dev)
        ptr = [[(act[t, g * n:(g + 1) * n].data_ptr(), obs[t + 1, g * n:(g + 1) * n].data_ptr(),
                 rew[t, g * n:(g + 1) * n].data_ptr()) for g in range(G)] for t in range(T)]
        o0 = [obs[0, g * n:(g + 1) * n].data_ptr() for g in range(G)]

        def episode(g, sp):
            e = envs[g]
            nat.check(e.lib.imenv_reset(e._h, None, nat.LAYOUT_DRAW, 0, 0.0, None, -1, o0[g], nat.F32, sp), "reset")
            for t in range(T):
                a, o, r = ptr[t][g]
                nat.check(e.lib.imenv_step(e._h, a, nat.F32, o, nat.F32, r, None, None, sp), "step")

        cur = torch.cuda.current_stream(dev)
        for g in range(G):            # warm: hipRTC build
            episode(g, streams[g].cuda_stream)
        torch.cuda.synchronize(dev)

        def eager_once():
            torch.cuda._sleep(3000000)        # ~ms: the host enqueues all G episodes behind it
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record(cur)
            for s in streams:
                s.wait_stream(cur)
            for g in range(G):
                episode(g, streams[g].cuda_stream)
            for s in streams:
                cur.wait_stream(s)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record(cur)
            ev1.synchronize()
            return ev0.elapsed_time(ev1) * 1e3 / T

        eager = sorted(eager_once() for _ in range(args.reps))[args.reps // 2]
        graph = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream(dev)
        with torch.cuda.graph(graph, stream=cs):
            c = torch.cuda.current_stream(dev)
            for s in streams:
                s.wait_stream(c)
            for g in range(G):
                episode(g, streams[g].cuda_stream)
            for s in streams:
                c.wait_stream(s)
        graph.replay()
        torch.cuda.synchronize(dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(cur)
        for _ in range(args.reps):
            graph.replay()
        ev1.record(cur)
        ev1.synchronize()
        gr = ev0.elapsed_time(ev1) * 1e3 / (args.reps * T)
        for mode, us in (("eager_queued", eager), ("graph", gr)):
            print(json.dumps({"mode": mode, "groups": G, "envs": total, "envs_per_group": n,
                              "us_per_step_incl_reset": round(us, 3),
                              "env_steps_per_s": round(total / (us * 1e-6), 1)}), flush=True)
        del graph
        for e in envs:
            e.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""The CPU port's speed against the reference itself, measured once here ("the
restatement/reference speed ratio is measured here once and recorded").

bench.py's cpu_baseline runs the oracle port (oracle/im_oracle.py) on the GPU box, where the reference
does not exist. This script, in the build container only, times the reference's own env classes
(imported with the same gym / RLlib stand-ins as tools/gen_fixtures.py: base classes only, no
arithmetic) and the port on the SAME episodes (host-fed Poisson(5) demand, uniform[-1, 1] actions as
float32 values, reset + 30 steps), one env per process as the reference runs under RLlib, one core
(CPU affinity), BLAS threads 1, alternating reference / port runs. Writes profiles/cpu_ratio.json;
bench.py quotes the ratio and the reference-equivalent rate beside its port baseline.

    python tools/cpu_ratio.py [--seconds 4] [--rounds 3]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "profiles", "cpu_ratio.json")
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-for-im_amd")]


def worker(which, cname, seconds, core):
    os.sched_setaffinity(0, {core})
    sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-for-im_amd"), os.path.join(ROOT, "tools")]
    import numpy as np
    import bench
    kind, cfg = bench.CONFIGS[cname][:2]
    rs = np.random.RandomState(1234)
    if which == "reference":
        from gen_fixtures import import_reference
        cls = import_reference()[kind]
        env = cls({k: (v.copy() if hasattr(v, "copy") else v) for k, v in cfg.items()})
        N = env.num_nodes if hasattr(env, "num_nodes") else env.num_stages
        serial = kind in ("IM", "MAIM")
        R = 1 if serial else len(env.retailers)
        names = None
        if kind == "MAIM":
            names = ["stage_%d" % i for i in range(N)]
        elif kind == "MAIM_div":
            names = ["node_%d" % i for i in range(N)]

        def episode(dem, act):
            env.reset(customer_demand=dem[0] if serial else dem)
            for t in range(30):
                a = act[t]
                env.step({nm: a[i:i + 1] for i, nm in enumerate(names)} if names else a)
    else:
        from oracle.im_oracle import OracleEnv
        env = OracleEnv(kind, cfg, n_envs=1)
        N, R = env.N, len(env.retailers)
        serial = kind in ("IM", "MAIM")

        def episode(dem, act):
            env.reset(customer_demand=dem[0][None, :] if serial else dem[None])
            for t in range(30):
                env.step(act[t][None, :])
    steps = 0
    t0 = time.perf_counter()
    while True:
        dem = rs.poisson(5, (R, 30))
        act = rs.uniform(-1, 1, size=(30, N)).astype(np.float32).astype(np.float64)
        episode(dem, act)
        steps += 30
        el = time.perf_counter() - t0
        if el >= seconds:
            return steps / el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--worker", nargs=3, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.worker:
        which, cname, core = args.worker
        print(json.dumps({"rate": worker(which, cname, args.seconds, int(core))}))
        return
    if not os.path.isdir("/root/reference"):
        raise SystemExit("cpu_ratio.py runs in the build container (the reference is not on the GPU box)")
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    out = {"what": "env-steps/s on ONE core, one env per process (reset + 30 steps, host-fed Poisson(5) demand, "
                   "uniform[-1,1] actions), BLAS threads 1; reference = environments/*.py imported with gym/RLlib "
                   "stand-ins (tools/gen_fixtures.py), port = oracle/im_oracle.py; median of alternating rounds",
           "host": os.uname().nodename, "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].split(":", 1)[1].strip(),
           "seconds_per_run": args.seconds, "rounds": args.rounds, "configs": {}}
    import statistics
    import bench
    for cname in ("C2", "C3", "C4"):
        rates = {"reference": [], "port": []}
        for _ in range(args.rounds):
            for which in ("reference", "port"):
                r = subprocess.run([sys.executable, os.path.abspath(__file__), "--seconds", str(args.seconds),
                                    "--worker", which, cname, "2"], env=env, capture_output=True, text=True,
                                   timeout=600)
                if r.returncode != 0:
                    raise SystemExit(r.stderr[-3000:])
                rates[which].append(json.loads(r.stdout.strip().splitlines()[-1])["rate"])
        ref, port = statistics.median(rates["reference"]), statistics.median(rates["port"])
        out["configs"][cname] = {"kind": bench.CONFIGS[cname][0], "reference_per_core": round(ref, 1),
                                 "port_per_core": round(port, 1), "port_over_reference": round(port / ref, 3),
                                 "runs": {k: [round(x, 1) for x in v] for k, v in rates.items()}}
        print(cname, out["configs"][cname], flush=True)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()

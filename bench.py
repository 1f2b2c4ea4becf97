#!/usr/bin/env python3
"""Throughput bench for the north-star path: env-steps/s of the HIP step kernel.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4] [--n-envs E]
                    [--scaling strong|weak] [--gather | --no-gather] [--no-cpu-baseline]

Workload (BASELINE.json metric "env-steps/sec (whole node), 4-stage x 2^20 envs"):
MultiAgentInvManagement, 4 stages, MA_1 flags (hyperparams.py:344; constants
inv_management.py:35-56), shared reward, 2^20 envs (global), 30-period episodes,
in-kernel Philox Poisson(5) demand, float32 actions pre-generated [30][n][4]
(torch.Generator seed 0) and float32 observations written into a [30][n][4][3]
rollout buffer, float64 rewards. A "step" = one step() of every env; the reset kernel
runs at each episode boundary, and the line's "resets_timed" says how many of them
fell inside the timed region.

Multi-GPU: one process per GPU. By default the ranks STRONG-scale the metric's 2^20 envs (BASELINE.json
configs[4]): rank r of W steps the contiguous global env ids shard_range(2^20, W, r), so
the 8-GPU line is C5 (8 x 131,072 envs) and --gpus 1 is the single-GPU metric workload; `--scaling
weak` gives every rank its own 2^20 envs instead. The ranks come either from an external launcher
(torchrun sets WORLD_SIZE / RANK / LOCAL_RANK) or, for `--gpus N` with no launcher, from this script
itself: the parent process starts N rank processes before it (or they) touch the GPU, and exits with
the first non-zero rank status. With N > 1 (or `--gather`) a second, separately timed pass adds C5's
per-step all-gather of obs+reward (RCCL over xGMI on the GPU node): the line's value and kernel time
come from the gather-free pass, the pipelined step+gather rate and the collective's own time are
reported under "gather".
The reference's own parallelism is one env per RLlib worker process (hyperparams.py:14,
MA_inv_management.py:172); the rank processes replace those workers.

Launch-bound batches (C5's 131,072-env shard, C3, C4: the host's per-step enqueue is a large part of the
kernel's time) run the timed K steps as one HIP graph captured before the timed region and replayed once
inside it (`--launch auto`, the default; `eager` / `graph` force one form); the metric's 2^20-env line is
launched eagerly, one host launch per step. roofline.launch_pacing says which form ran.

Prints ONE JSON line on rank 0 (keys per the driver contract), with "roofline" (step
kernel: algorithmic bytes / HIP-event-timed kernel duration vs 8 TB/s; plus an
informational HIP-graph-replayed episode) and "cpu_baseline" (the oracle port, one env
per process, timed on this box's host cores before the GPU is touched).
"""
import argparse
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "marl-for-im_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

METRIC = "env-steps/sec (whole node), 4-stage × 2^20 envs; % HBM roofline"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table: 8.0 TB/s HBM3E (spec)
CPU_SHARE = 16             # host cores per GPU on the GPU box (worker pools must stay within it)
CPU_BASELINE_ENV = "IMENV_BENCH_CPU_BASELINE"   # launcher -> rank 0: the CPU baseline it measured

C2_CONFIG = dict(num_stages=4, num_periods=30, init_inv=np.ones(4) * 10, inv_target=np.zeros(4),
                 inv_max=np.ones(4) * 30, price=np.array([5, 4, 3, 2, 1]),
                 stock_cost=np.array([0.35, 0.3, 0.4, 0.2]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.9]),
                 delay=np.array([1, 2, 3, 1], dtype=np.int8), demand_dist="poisson", mu=5, seed=52,
                 standardise_state=True, standardise_actions=True, a=-1, b=1, time_dependency=False,
                 prev_demand=False, prev_actions=False, prev_length=1, independent=False)


C3_CONFIG = dict(num_stages=8, num_periods=30, init_inv=np.ones(8) * 10, inv_target=np.zeros(8),
                 inv_max=np.ones(8) * 30, price=np.array([9, 8, 7, 6, 5, 4, 3, 2, 1]),
                 stock_cost=np.array([0.35, 0.3, 0.4, 0.2, 0.35, 0.3, 0.4, 0.2]),
                 backlog_cost=np.array([0.5, 0.7, 0.6, 0.9, 0.5, 0.7, 0.6, 0.9]),
                 delay=np.array([1, 2, 3, 1, 4, 2, 3, 1]), demand_dist="poisson", mu=5, seed=52)
C4_CONFIG = dict(num_nodes=4, connections={0: [1], 1: [2, 3], 2: [], 3: []}, num_periods=30,
                 init_inv=np.ones(4) * 10, inv_target=np.zeros(4), inv_max=np.ones(4) * 30,
                 stock_cost=np.array([0.35, 0.3, 0.4, 0.4]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.6]),
                 delay=np.array([1, 2, 1, 1]), demand_dist="poisson", mu=5, seed=52, time_dependency=True,
                 prev_demand=True, prev_actions=False, prev_length=1, independent=False)
# name -> (env kind, config, description, BASELINE.json size). C2 at 2^20 envs is the metric's workload
# (the default); C3 / C4 are BASELINE's other single-GPU configs (parity cases; --config selects them)
CONFIGS = {
    "C2": ("MAIM", C2_CONFIG, "MultiAgentInvManagement 4-stage serial (inv_management.py:35-56 constants, "
                              "MA_1 flags, shared reward)", 1 << 20),
    "C3": ("IM", C3_CONFIG, "InvManagement 8-stage serial chain (SHLP_8.py:26-46 constants, flags off)", 262144),
    "C4": ("MAIM_div", C4_CONFIG, "MultiAgentInvManagementDiv div1 2-retailer tree (MA_inv_management_div.py:46-69, "
                                  "MA_6 flags: time_dependency + prev_demand L=1, shared reward)", 131072),
}


# ----------------------------------------------------------------- CPU baseline
def _cpu_worker(args):
    seconds, seed, cname = args
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle.im_oracle import OracleEnv
    kind, cfg = CONFIGS[cname][:2]
    rs = np.random.RandomState(seed)
    env = OracleEnv(kind, cfg, n_envs=1)
    N, R = env.N, len(env.retailers)
    steps = 0
    t0 = time.perf_counter()
    while True:
        dem = rs.poisson(5, 30) if kind in ("IM", "MAIM") else rs.poisson(5, (1, R, 30))
        act = rs.uniform(-1, 1, size=(30, 1, N)).astype(np.float32).astype(np.float64)
        env.reset(customer_demand=dem)
        for t in range(30):
            env.step(act[t])
        steps += 30
        el = time.perf_counter() - t0
        if el >= seconds:
            return steps, el


def cpu_baseline(seconds=1.5, cname="C2"):
    """Oracle port of the reference step(), one env per process (the reference's own usage:
    one env per RLlib worker), a pool over this box's cores. Runs in a child interpreter
    started with BLAS threads pinned to 1 (they must be set before numpy is imported)."""
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-only", "--cpu-seconds", str(seconds),
                        "--config", cname],
                       env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError("cpu baseline failed: " + r.stderr[-2000:])
    out = json.loads(r.stdout.strip().splitlines()[-1])
    # the port's speed relative to the reference's own step(), measured once where the reference exists
    # (tools/cpu_ratio.py: one core, the same episodes), so the line can say what the
    # reference itself would do on these cores
    try:
        with open(os.path.join(ROOT, "profiles", "cpu_ratio.json")) as f:
            ratio = float(json.load(f)["configs"][cname]["port_over_reference"])
        out.update(port_over_reference=ratio, reference_equiv_value=round(out["value"] / ratio, 1),
                   ratio_source="profiles/cpu_ratio.json: the reference's environments/*.py step() and this port "
                                "timed on the same episodes, one core, in the build container (tools/cpu_ratio.py)")
    except (OSError, KeyError, ValueError):
        pass
    return out


def _cpu_baseline_here(seconds, cname):
    # the GPU box's CPU share is 16 cores per GPU (os.cpu_count() there reports the whole host, many
    # times that, and larger pools are refused); both numbers go into the sample text
    visible = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cores = max(1, min(CPU_SHARE, visible))
    ctx = mp.get_context("fork")   # before any GPU call in this process: plain fork, no exec
    with ctx.Pool(cores) as pool:
        res = pool.map(_cpu_worker, [(seconds, 100 + i, cname) for i in range(cores)])
    total = sum(s / e for s, e in res)
    return dict(value=round(total, 1), unit="env-steps/s", cores=cores, kind="port",
                sample="oracle/im_oracle.py %s (%s config), 1 env per process, %d processes x "
                       "%.1f s of whole 30-period episodes each (%d env-steps total), host-fed Poisson(5) demand, "
                       "BLAS threads 1; per core %.0f env-steps/s; pool capped at the box's %d-core CPU share "
                       "per GPU (host reports %d visible, %d total)"
                       % (CONFIGS[cname][0], cname, cores, seconds, sum(s for s, _ in res), total / cores,
                          CPU_SHARE, visible, os.cpu_count()))


# ----------------------------------------------------------------- PMC traffic
def pmc_record(n_envs, kernel):
    """The committed rocprofv3 summary of this exact kernel variant (kernel_info) at this size:
    profiles/pmc_step_kernel.json (written by tools/profile_pmc.sh) or profiles/pmc_configs/*.json
    (tools/profile_configs.sh: PMC passes + the kernel trace of the same bench command), else None.
    A diagnostic build (tag "jit-diag:") never matches."""
    import glob
    if kernel.startswith("jit-diag:"):
        return None
    paths = [os.path.join(ROOT, "profiles", "pmc_step_kernel.json")]
    paths += sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_configs", "*.json")))
    for p in paths:
        try:
            with open(p) as f:
                d = json.load(f)
            if int(d.get("n_envs", -1)) == int(n_envs) and d.get("kernel_info") == kernel:
                d["_path"] = os.path.relpath(p, ROOT)
                return d
        except Exception:
            continue
    return None


def pmc_traffic(n_envs, kernel):
    """HBM bytes per step-kernel launch from the committed PMC summary of this kernel variant, else None."""
    d = pmc_record(n_envs, kernel)
    return float(d["hbm_bytes_per_launch"]) if d and "hbm_bytes_per_launch" in d else None


# ----------------------------------------------------------------- HIP events
class HipEvent:
    """A timing event of the HIP runtime torch itself loaded (libamdhip64.so.7, one copy per process),
    recorded through ctypes: ~1 us of host time per record against ~10-20 us for torch.cuda.Event.record,
    which the timed region of a small launch (3.6 us per step at 131,072 envs) cannot afford."""
    _lib = None

    @classmethod
    def lib(cls):
        if cls._lib is None:
            import ctypes
            lib = ctypes.CDLL("libamdhip64.so.7")
            lib.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
            lib.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            lib.hipEventSynchronize.argtypes = [ctypes.c_void_p]
            lib.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
            lib.hipEventDestroy.argtypes = [ctypes.c_void_p]
            cls._lib = lib
        return cls._lib

    def __init__(self):
        import ctypes
        self.h = ctypes.c_void_p()
        if self.lib().hipEventCreate(ctypes.byref(self.h)) != 0:
            raise RuntimeError("hipEventCreate failed")
        self._rec = self._lib.hipEventRecord
        self.hv = self.h.value

    def record(self, stream_ptr):
        if self._rec(self.hv, stream_ptr) != 0:
            raise RuntimeError("hipEventRecord failed")

    def elapsed_time(self, end):
        """ms from this event to `end` (both completed)."""
        import ctypes
        self._lib.hipEventSynchronize(end.hv)
        ms = ctypes.c_float()
        if self._lib.hipEventElapsedTime(ctypes.byref(ms), self.hv, end.hv) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return ms.value

    def __del__(self):
        try:
            self._lib.hipEventDestroy(self.hv)
        except Exception:
            pass


# ----------------------------------------------------------------- launcher
def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv):
    """`--gpus N` (N > 1) with no launcher: start N rank processes of this script, one per GPU, from a
    process that has not touched the GPU (no exec: children, whose exit codes this one returns). Rank 0
    prints the line. The CPU baseline runs here first, on the host cores, and is handed to rank 0."""
    n = args.gpus
    cpu = None
    if not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds, args.config)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, WORLD_SIZE=str(n), RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), IMENV_BENCH_LAUNCHER="self")
        if cpu is not None:
            env[CPU_BASELINE_ENV] = json.dumps(cpu)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    alive = list(procs)
    while alive:
        time.sleep(0.05)
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                sys.stderr.write("bench.py: rank process %d exited with %d; stopping the others\n" % (p.pid, code))
                for q in alive:
                    q.terminate()
    sys.exit(rc)


def ranks_census(dist, dev):
    """Every rank's (rank, local rank, device, PCI bus id): the line reports how many distinct ranks and
    GPUs took part, so a line cannot claim N GPUs while fewer ran."""
    import torch
    me = {"rank": dist.get_rank() if dist.is_initialized() else 0,
          "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "host": socket.gethostname()}
    if dev is not None:
        pr = torch.cuda.get_device_properties(dev)
        me.update(device=dev.index, gpu="%04x:%02x:%02x" % (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id))
    if not dist.is_initialized():
        return [me]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, me)
    return out


def shard_plan(scaling, config, n_envs, world, rank):
    """(global env id of this rank's first env, envs on this rank, global envs of the job).

    strong (default): the job steps n_envs global envs (default: the config's BASELINE.json size, 2^20
    for C2) and rank r owns the contiguous ids shard_range(n_envs, world, r); so with 8
    ranks the C2 line is BASELINE's C5, 8 x 131,072 envs. weak: every rank owns n_envs envs of its own,
    at ids [r * n_envs, (r + 1) * n_envs)."""
    from imenv.shard import shard_range, weak_offset
    total = int(n_envs or CONFIGS[config][3])
    if scaling == "strong":
        off, n = shard_range(total, world, rank)
        return off, n, total
    return weak_offset(total, rank), total, total * world


def episode_phase(W, K, T):
    """Period of the bench's step 0: step s runs period (s + phase) mod T. With K >= T every window of K
    steps holds a reset anyway (phase 0). A shorter window (the driver's --steps 20 --warmup 5) is placed so
    that the episode boundary falls in its middle: the timed steps then include a reset kernel, as they do
    on average in a long run (the reset runs every 30 steps inside the timed loop). The
    handle is brought to that period by untimed steps before the warmup."""
    return 0 if K >= T else (-(W + K // 2)) % T


def resets_in_window(W, K, T, phase):
    """Reset kernels inside the timed steps W .. W+K-1 (one before each period-0 step)."""
    return sum(1 for s in range(W, W + K) if (s + phase) % T == 0)


def gather_is_on(args, world):
    """The per-step all-gather leg: explicit --gather / --no-gather, else on whenever there is more than
    one rank (C5: the obs / reward batch gathered over xGMI)."""
    return args.gather if args.gather is not None else world > 1


def dry_run(args, world, rank):
    """The launcher / rendezvous / census / max-reduction path with no GPU work (CPU tests, gloo): the
    line carries n_gpus, ranks_seen and the shard plan, value null. With the gather leg on, StepGather
    runs over CPU tensors with gloo for K steps (every rank writes values derived from its global env
    ids and each step; every gathered step is checked) and gather_report is computed as on the GPU."""
    import torch
    import torch.distributed as dist
    if os.environ.get("IMENV_BENCH_DRY_FAIL_RANK") == str(rank):     # tests: a rank that dies
        sys.exit(7)
    if world > 1:
        dist.init_process_group("gloo")
    census = ranks_census(dist, None)
    off, n, total = shard_plan(args.scaling, args.config, args.n_envs, world, rank)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    gather_info = None
    if gather_is_on(args, world) and world > 1:
        gather_info = dry_gather(args, dist, world, n, off, total)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "env-steps/s", "n_gpus": world,
                          "dry_run": True, "ranks_seen": len({c["rank"] for c in census}), "ranks": census,
                          "max_over_ranks": t.item(), "launcher": os.environ.get("IMENV_BENCH_LAUNCHER", "external"),
                          "scaling": args.scaling,
                          "config": {"n_envs_per_gpu": n, "global_envs": total, "env_offset": off},
                          "gather": gather_info,
                          "cpu_baseline": json.loads(os.environ[CPU_BASELINE_ENV])
                          if CPU_BASELINE_ENV in os.environ else None}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def dry_gather(args, dist, world, n, off, total):
    """StepGather's double-buffered pipeline as bench.py drives it (write into obs_out(s) /
    reward_out(s), start(s), result(s-1)) on CPU tensors with gloo. The dry run's shards must be equal
    (the all-gather needs one shape on every rank)."""
    import torch
    from imenv.shard import StepGather
    N, F = 4, 3
    if total % world:
        raise SystemExit("dry-run gather: %d envs do not split evenly over %d ranks" % (total, world))
    ids = torch.arange(off, off + n, dtype=torch.float64)
    g = StepGather(torch.empty((n, N, F), dtype=torch.float32), torch.empty((n,), dtype=torch.float64))
    allids = torch.arange(total, dtype=torch.float64)

    def check(s):
        o, r = g.result(s)
        want_r = allids * 1000 + s
        if not (torch.equal(r, want_r) and torch.equal(o[:, 0, 0], (allids % 4096 + s).float())):
            raise SystemExit("dry-run gather: step %d gathered the wrong values" % s)

    steps = args.steps
    g.keep_works(True)
    for s in range(steps):
        g.obs_out(s).fill_(0.0)[:, 0, 0] = (ids % 4096 + s).float()
        g.reward_out(s).copy_(ids * 1000 + s)
        g.start(s)
        if s > 0:
            check(s - 1)
    check(steps - 1)
    return gather_report(g, dist, None, None, steps, world, n)


# ----------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=60)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS),
                    help="C2 (default): the metric's workload; C3 / C4: BASELINE's other single-GPU configs")
    ap.add_argument("--n-envs", type=int, default=None,
                    help="envs of the whole job under strong scaling, per GPU under weak scaling (default: "
                         "2^20 for C2, BASELINE.json's size for C3 / C4)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong (default): the ranks split --n-envs global envs; weak: every rank owns --n-envs")
    ap.add_argument("--weak", dest="scaling", action="store_const", const="weak", help="same as --scaling weak")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--gather", dest="gather", action="store_true", default=None,
                    help="time the per-step all-gather of obs+reward in a second pass (default: on with >1 rank)")
    ap.add_argument("--no-gather", dest="gather", action="store_false")
    ap.add_argument("--store", default="default", choices=["default", "stream", "plain", "writethrough"],
                    help="store policy of the step kernel (imenv_set_store_policy)")
    ap.add_argument("--no-alt-store", action="store_true", help="skip the informational run of the other policy")
    ap.add_argument("--no-graph", action="store_true", help="skip the informational HIP-graph episode replay")
    ap.add_argument("--launch", default="auto", choices=["auto", "eager", "graph"],
                    help="how the timed K steps reach the GPU: one host launch per step (eager), or the K steps "
                         "captured beforehand into one HIP graph and replayed once (graph); auto: graph where the "
                         "host's per-step enqueue is at least 30%% of the kernel (launch-bound small batches)")
    ap.add_argument("--no-alt-obs", action="store_true", help="skip the informational float64-observation run")
    ap.add_argument("--cpu-only", action="store_true", help=argparse.SUPPRESS)
    # rehearsal of the multi-rank path on a one-GPU box: every rank on device 0, gloo for the
    # barrier / max-reduction (the driver's N-GPU runs use one GPU per rank and RCCL)
    ap.add_argument("--rehearse-one-gpu", action="store_true", help=argparse.SUPPRESS)
    # the RCCL path of an N-rank line at world size 1 on one GPU: a one-rank "nccl" process group, the
    # census, barriers and max-reductions through it and the gather pass over RCCL (validation only)
    ap.add_argument("--rccl-solo", action="store_true", help=argparse.SUPPRESS)
    # launcher / rendezvous / census path only, no GPU work (CPU tests)
    ap.add_argument("--dry-run", action="store_true", help=argparse.SUPPRESS)
    argv = sys.argv[1:]
    args = ap.parse_args(argv)
    if args.steps < 1 or args.warmup < 0 or args.gpus < 1:
        ap.error("--steps must be >= 1, --warmup >= 0, --gpus >= 1")
    if args.cpu_only:
        print(json.dumps(_cpu_baseline_here(args.cpu_seconds, args.config)))
        return

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        launch_ranks(args, argv)          # never returns
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.stderr.write("bench.py: --gpus %d but the launcher started %d ranks\n" % (args.gpus, world))
        sys.exit(2)
    if args.dry_run:
        dry_run(args, world, rank)
        return

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        if CPU_BASELINE_ENV in os.environ:      # measured by this script's own launcher before the ranks started
            cpu = json.loads(os.environ[CPU_BASELINE_ENV])
        else:
            cpu = cpu_baseline(args.cpu_seconds, args.config)          # before the GPU is initialised

    if args.rccl_solo and (world != 1 or args.rehearse_one_gpu):
        sys.stderr.write("bench.py: --rccl-solo is the one-rank RCCL check (world size 1, no rehearsal)\n")
        sys.exit(2)
    dist_on = world > 1 or args.rccl_solo     # a process group (and its collectives) in this run
    gather_on = (gather_is_on(args, world) and world > 1) or (args.rccl_solo and args.gather is not False)
    if gather_on and not args.rehearse_one_gpu:
        # RCCL records start / end events around every collective on its own stream (Work._get_duration)
        os.environ.setdefault("TORCH_NCCL_ENABLE_TIMING", "1")
        # ... and takes those events from a cache: an event of an eager collective that the watchdog still
        # polls could come back recorded in the capturing stream of the graph-captured gather pass, and
        # the watchdog's query then aborts the process ("operation not permitted on an event last recorded
        # in a capturing stream"): fresh events per collective
        os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    import torch
    import torch.distributed as dist
    from imenv import VectorInvEnv
    from imenv import _native as nat
    from imenv.shard import StepGather

    if args.rehearse_one_gpu:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist_on:
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo")
        else:
            if args.rccl_solo:
                for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", str(_free_port())), ("RANK", "0"),
                             ("WORLD_SIZE", "1")):
                    os.environ.setdefault(k, v)
            dist.init_process_group("nccl", device_id=dev)
    census = ranks_census(dist, dev)
    ranks_seen = len({c["rank"] for c in census})
    gpus_seen = len({(c["host"], c["gpu"]) for c in census})
    if ranks_seen != world:
        sys.stderr.write("bench.py: %d ranks took part, world size is %d\n" % (ranks_seen, world))
        sys.exit(3)

    kind, ccfg, cdesc, _ = CONFIGS[args.config]
    env_off, n, global_envs = shard_plan(args.scaling, args.config, args.n_envs, world, rank)
    env = VectorInvEnv(kind, ccfg, n_envs=n, device=dev, env_offset=env_off)
    N, F, T = env.N, env.F, env.T
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    actions = torch.rand((T, n, N), generator=g, device=dev, dtype=torch.float32) * 2 - 1
    obs_buf = torch.empty((T, n, N, F), dtype=torch.float32, device=dev)
    obs0 = torch.empty((n, N, F), dtype=torch.float32, device=dev)
    rew_buf = torch.empty((T,) + env.reward_shape(), dtype=torch.float64, device=dev)

    lib, h = env.lib, env._h
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    a_ptr = [actions[t].data_ptr() for t in range(T)]
    o_ptr = [obs_buf[t].data_ptr() for t in range(T)]
    r_ptr = [rew_buf[t].data_ptr() for t in range(T)]

    def reset(sp):
        nat.check(lib.imenv_reset(h, None, nat.LAYOUT_DRAW, 0, 0.0, None, -1, obs0.data_ptr(), nat.F32, sp),
                  "imenv_reset")

    # HIP events on the kernel's own stream bracket every run of consecutive step launches between two
    # resets (at most one episode, and the part of one that the timed region holds): per-launch
    # duration = elapsed / launches of the run, back-to-back dispatch gaps included, the reset kernel
    # outside every pair. Every timed step launch lies in exactly one pair, whatever K and W are. One
    # pair per episode: a pair per step would cost ~7 us of GPU time each and slow the very loop
    # being measured (tools/launch_probe.py). The event pairs are only ever used on the gather-free
    # pass, so no collective wait lies between them.
    obs64 = {}     # float64 observation buffers of the informational alt_obs_f64 leg (made on demand)

    def run(first, steps, events=None, gather=None, f64=False, sp=None, resets_here=True):
        """Steps first .. first+steps-1 of the bench's step sequence (period t = (step + phase) mod T). With a
        StepGather the env writes into its send buffers and step s's all-gather runs under step s+1;
        with f64 the observations are float64 (the reference's dtype). Returns the number of resets it
        ran."""
        pair = None
        resets = 0
        op, od = (obs64["ptr"], nat.F64) if f64 else (o_ptr, nat.F32)
        step, F32 = lib.imenv_step, nat.F32      # (locals: the loop is host-paced at small launches)
        sptr_ = sptr if sp is None else sp       # the stream the steps go to (a capture stream for graphs)
        for s in range(first, first + steps):
            t = (s + phase) % T
            if t == 0 and resets_here:
                reset(sptr_)
                resets += 1
            if events is not None and pair is None:
                pair = [pool.pop(), pool.pop(), []]     # pre-created in timed()
                pair[0].record(sptr_)
            if pair is not None:
                pair[2].append(t)
            if gather is None:
                rc = step(h, a_ptr[t], F32, op[t], od, r_ptr[t], None, None, sptr_)
            else:
                # the env writes straight into the packed send buffer of step s (double-buffered); the
                # all-gather of step s runs on the collective's stream under step s+1
                rc = lib.imenv_step(h, a_ptr[t], nat.F32, gather.obs_out(s).data_ptr(), nat.F32,
                                    gather.reward_out(s).data_ptr(), None, None, sptr_)
            if rc:
                nat.check(rc, "imenv_step")
            if pair is not None and (t == T - 1 or s == first + steps - 1):
                pair[1].record(sptr_)
                events.append(pair)
                pair = None
            if gather is not None:
                gather.start(s)
                if s > first:
                    gather.result(s - 1)     # the learner's view of step s-1: [global n, N, F], [global n]
        if gather is not None and steps:
            gather.result(first + steps - 1)
        return resets

    per_t = env.step_traffic_per_period()
    per_t64 = env.step_traffic_per_period(obs_bytes=8)

    def lead_spin(W, K, f64=False):
        """GPU cycles of a busy-wait (torch.cuda._sleep) to enqueue ahead of the timed launches. Small
        launches (C4 at 131,072 envs: ~5.6 us each) are shorter than the host's enqueue of one step
        (~6 us of Python, ctypes and hipModuleLaunchKernel), so the GPU would idle between launches and
        the event pairs would time the host's pace instead of the kernel's. A spin as long as the host
        falls behind over the K steps lets the launches queue up, so the events time them back to back;
        the wall-clock value is unchanged up to the 5% margin on that spin (the host paces the loop
        either way: the last launch still follows the host's last enqueue). When the host keeps
        well ahead (the metric's 2^20-env launches), no spin; when it keeps ahead by a thin margin, a
        short fixed lead (below). Calibrated on two untimed episodes (the step
        sequence stays aligned: 2T steps bring the handle back to the same period). Returns (cycles,
        host us per step, GPU us per step)."""
        if not hasattr(torch.cuda, "_sleep"):    # (a private torch helper: without it, no pacing)
            return 0, float("nan"), float("nan")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        e0.record(stream)
        torch.cuda._sleep(200000)
        e1.record(stream)
        e1.synchronize()
        us_per_cycle = e0.elapsed_time(e1) * 1e3 / 200000
        us_per_cycle_cal[:] = [us_per_cycle]
        n_cal = 2 * T
        torch.cuda._sleep(int(3000 / us_per_cycle))       # 3 ms: longer than enqueueing n_cal steps
        e0.record(stream)
        hs = []
        for k in range(2):          # two episodes, the faster host pace counts (a descheduled host
            h0 = time.perf_counter()    # thread in one of them must not buy a long spin)
            run(W + k * T, T, f64=f64)
            hs.append((time.perf_counter() - h0) * 1e6 / T)
        h = min(hs)
        e1.record(stream)
        e1.synchronize()
        g = e0.elapsed_time(e1) * 1e3 / n_cal
        if os.environ.get("IMENV_BENCH_LEAD_US"):      # experiments: a forced lead (us) ahead of the K launches
            return int(float(os.environ["IMENV_BENCH_LEAD_US"]) / us_per_cycle), h, g
        if h > g:
            return int(K * (h - g) * 1.05 / us_per_cycle), h, g
        if h > 0.6 * g:
            # the host keeps ahead, but by less than 40% of a launch: one late enqueue (a scheduler or
            # allocator hiccup of tens of us) would leave the GPU idle inside an event pair. A fixed lead
            # of min(10% of the K launches, 50 us) absorbs it; the wall clock pays that lead in full
            return int(min(0.1 * K * g, 50.0) / us_per_cycle), h, g
        return 0, h, g

    spin_info = {}
    window_info = {}
    graph_span = []            # launch=graph: [span ms, resets, periods of the timed steps]
    reset_cache = []

    def reset_alone_us():
        """The reset kernel alone (us per launch): 20 back-to-back resets queued behind a busy-wait, HIP events
        on the kernel's stream. Leaves the handle at period 0 (every timed() pass re-positions it)."""
        if not reset_cache:
            torch.cuda.synchronize(dev)
            r0, r1 = HipEvent(), HipEvent()
            torch.cuda._sleep(2000000)
            r0.record(sptr)
            for _ in range(20):
                reset(sptr)
            r1.record(sptr)
            reset_cache.append(r0.elapsed_time(r1) * 1e3 / 20)
        return reset_cache[0]
    us_per_cycle_cal = []      # GPU busy-wait cycles -> us (lead_spin's calibration)

    def bracket(body):
        """The driver's timed region: barrier + synchronise, then body(), then synchronise; the wall time
        is read before the trailing barrier (every rank's own K steps, not the slowest rank's barrier
        exit), and the max over ranks is taken afterwards."""
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        out = body()
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        el = t2 - t0
        if dist_on:
            dist.barrier()
        # where the window's wall time went (host side): enqueueing the K steps, then waiting for the GPU
        window_info.update(host_enqueue_us=round((t1 - t0) * 1e6, 1), sync_wait_us=round((t2 - t1) * 1e6, 1))
        return el, out

    def max_over_ranks(*xs):
        if not dist_on:
            return xs
        tt = torch.tensor(list(xs), dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return tuple(v.item() for v in tt)

    def warm(W, **kw):
        """Bring the handle to step W of the sequence: a reset and the untimed steps of periods 0 ..
        phase - 1 (episode_phase), then the W warmup steps."""
        if W == 0:
            run(-phase, 1, **kw)     # no warmup asked for: one step outside the sequence builds the hipRTC kernel
        run(-phase, phase + W, **kw)

    def timed(W, K, f64=False):
        """W untimed warmup steps, then exactly K timed steps of the same step sequence, so the timed
        region holds the resets at its episode boundaries (at least one: episode_phase). No collective.
        Returns (wall s, kernel ms per launch, algorithmic bytes per timed launch, timed launches, resets
        timed), max over ranks."""
        warm(W, f64=f64)
        spin, h_us, g_us = lead_spin(W, K, f64)
        # auto: a graph where the host's per-step enqueue (measured with the GPU idle) is at least 30% of the
        # GPU's per-step time; with the GPU running, the host's enqueue takes up to twice as long (kernel
        # arguments written over PCIe into device memory), so an eager window of such launches is host-paced
        # (C4 at 131,072 envs: 3.3 vs 5.8 us per step, eager kernel_us 9.0 in the driver's window)
        graph = args.launch == "graph" or (args.launch == "auto" and h_us == h_us and h_us > 0.3 * g_us)
        if not spin_info:      # the line's own timed region (not the informational alt-store run)
            spin_info.update(host_us_per_step=None if h_us != h_us else round(h_us, 3),
                             gpu_us_per_step_queued=None if g_us != g_us else round(g_us, 3),
                             lead_spin_cycles=0 if graph else spin, launch="graph" if graph else "eager")
        # the timed region's event pairs (raw HIP events: HipEvent), created and recorded once before it
        # starts: one pair per run of steps between resets
        pool[:] = [HipEvent() for _ in range(2 * (K // T + 2))]
        for e in pool:
            e.record(sptr)
        torch.cuda.synchronize(dev)
        events = []
        span_ms = None
        if graph:
            # launch-bound small batches (C5's 131,072-env shard: 3.3-9 us of host work per launch against
            # 3.6-3.8 us of kernel, so an eager window is paced by the host): the same K steps and resets,
            # captured into ONE HIP graph before the timed region (the handle's host period advances at
            # capture, its device state at replay) and replayed once inside it. Same kernels, same arguments,
            # same order; the host submits them in one call. HIP events recorded inside a captured graph do
            # not time reliably here, and one graph per run of steps between resets costs ~10 us of GPU-side
            # gap per replay (both measured: profiles/r05/launch_modes/), so the kernel time is the span of
            # events around the replay minus the window's resets (reset_us, timed alone in this run), over K.
            # A 20 us busy-wait lead lets the host submit the graph before the GPU reaches the first event.
            cur = torch.cuda.current_stream(dev).cuda_stream
            cs = torch.cuda.Stream(dev)
            gph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gph, stream=cs):
                resets = run(W, K, f64=f64, sp=torch.cuda.current_stream(dev).cuda_stream)
            torch.cuda.synchronize(dev)
            ga, gb = HipEvent(), HipEvent()
            lead = int(20.0 / us_per_cycle_cal[0]) if us_per_cycle_cal else 0

            def replay():
                if lead:
                    torch.cuda._sleep(lead)
                ga.record(cur)
                gph.replay()
                gb.record(cur)
            el, _ = bracket(replay)
            span_ms = ga.elapsed_time(gb)
            del gph
            ts = [(W + k + phase) % T for k in range(K)]
            graph_span[:] = [span_ms, resets, ts]
        else:
            def body():
                if spin:
                    torch.cuda._sleep(spin)
                return run(W, K, events, f64=f64)
            el, resets = bracket(body)
        if graph:
            launches = K
            kern_ms = None            # (span - resets x reset_us) / K once the reset is timed (below)
            first_last = span_ms
            ksrc = ("HIP events around the one graph replay of the window, minus resets_timed x reset_us, over K "
                    "(launch=graph)")
            bpl = sum((per_t64 if f64 else per_t)[t] for t in graph_span[2]) * n / K
        else:
            launches = sum(len(ts) for _, _, ts in events)
            kern_ms = sum(a.elapsed_time(b) for a, b, _ in events) / launches
            first_last = events[0][0].elapsed_time(events[-1][1])
            ksrc = "HIP event pairs around each run of step launches between resets"
        if not spin_info.get("window"):      # the line's own timed region
            spin_info["window"] = dict(window_info, gpu_span_us=round(first_last * 1e3, 1), wall_us=round(el * 1e6, 1),
                                       kernel_us_source=ksrc)
        # per-launch kernel time and the algorithmic bytes of exactly the launches that were timed
        pt = per_t64 if f64 else per_t
        if not graph:
            bpl = sum(pt[t] for _, _, ts in events for t in ts) * n / launches
        if kern_ms is None:
            rus = reset_alone_us()
            kern_ms = (span_ms - resets * rus * 1e-3) / K
            spin_info["window"]["reset_us_subtracted"] = round(resets * rus, 3)
        el, kern_ms = max_over_ranks(el, kern_ms)
        return el, kern_ms, bpl, launches, resets

    def timed_gather(W, K, gather):
        """The same W + K step sequence with C5's per-step all-gather pipelined under the next step (a
        second pass after the line's own): the wall time of the K steps including every collective, max
        over ranks."""
        warm(W, gather=gather)
        gather.keep_works(True)
        el, _ = bracket(lambda: run(W, K, gather=gather))
        return max_over_ranks(el)[0]

    pool = []
    W, K = args.warmup, args.steps
    phase = episode_phase(W, K, T)
    env.set_store_policy(args.store)
    el, kern_ms, bytes_per_launch, launches, resets_timed = timed(W, K)
    kinfo = env.kernel_info()          # the timed kernel (before the informational runs below)

    # the reset kernel alone (the line's value already holds resets_timed of them): 20 back-to-back
    # resets queued behind a busy-wait, HIP events on the kernel's stream
    reset_us = reset_alone_us() if hasattr(torch.cuda, "_sleep") else None

    gather_info = None
    if gather_on and args.scaling == "strong" and global_envs % world:
        # all_gather_into_tensor needs one send size on every rank; uneven shards would hand RCCL
        # different counts (undefined behaviour: a hang or a corrupt buffer, not an exception)
        gather_on = False
        gather_info = {"skipped": "%d envs do not split evenly over %d ranks: the all-gather needs equal shards"
                                  % (global_envs, world)}
    if gather_on:
        backend = dist.get_backend()
        try:
            gth = StepGather(obs_buf[0], rew_buf[0])
            g_el = timed_gather(W, K, gth)
            gather_info = gather_report(gth, dist, dev, stream, K, world, n)
            gather_info.update(backend="gloo (one-GPU rehearsal)" if args.rehearse_one_gpu else
                               "%s (RCCL over xGMI)" % backend if backend == "nccl" else backend,
                               pipelined_value=round(global_envs * K / g_el, 1),
                               pipelined_ms_per_step=round(g_el / K * 1e3, 6),
                               pipelined_over_gather_free=round(el / g_el, 4),
                               pipelined_form="eager: one host launch per step and per collective")
            if backend == "nccl" and world == 1:
                # the same pipeline with the host out of the loop: one episode's reset, T steps and T
                # all-gathers captured into one HIP graph and replayed. One rank only (--rccl-solo): with
                # more ranks the per-step collective is bound by the xGMI links (58.7 MB received per rank
                # per step at N = 8), not by the host, and a capture that failed on one rank while the
                # others replayed would leave their collectives waiting for it
                try:
                    gg = graph_gather_run(torch, dist, dev, gth, reset, lib, nat, a_ptr, T, h)
                    gather_info["graph"] = gg
                    if gg["ms_per_step"] * 1e-3 < g_el / K:
                        gather_info["eager"] = {k: gather_info[k] for k in ("pipelined_value", "pipelined_ms_per_step",
                                                                             "pipelined_over_gather_free")}
                        gather_info.update(pipelined_value=round(global_envs / (gg["ms_per_step"] * 1e-3), 1),
                                           pipelined_ms_per_step=gg["ms_per_step"],
                                           pipelined_over_gather_free=round(el / K / (gg["ms_per_step"] * 1e-3), 4),
                                           pipelined_form="HIP graph: reset + %d steps + %d all-gathers per replay "
                                                          "(gather.graph), the eager form under gather.eager" % (T, T))
                except Exception as ex:
                    gather_info["graph"] = {"error": "%s: %s" % (type(ex).__name__, str(ex)[:300])}
            del gth
        except Exception as ex:          # informational leg: the line still reports the gather-free pass
            gather_info = {"error": "%s: %s" % (type(ex).__name__, str(ex)[:300])}

    alt = None
    if world == 1 and not args.no_alt_store:
        # another store policy on the same handle (informational; the line's value is args.store's):
        # plain cached stores (round 2's default) next to the default, else the default
        other = "plain" if args.store == "default" else "default"
        env.set_store_policy(other)
        a_el, a_kern, a_bpl, _, _ = timed(W, K)
        a_kinfo = env.kernel_info()
        env.set_store_policy(args.store)
        alt = {"store_policy": other, "kernel": a_kinfo, "value": round(n * K / a_el, 1),
               "ms_per_step": round(a_el / K * 1e3, 6),
               "kernel_us": round(a_kern * 1e3, 3), "achieved": round(a_bpl / (a_kern * 1e-3) / 1e9, 1),
               "frac": round(a_bpl / (a_kern * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}

    alt64 = None
    if world == 1 and not args.no_alt_obs:
        # the reference's observation dtype (float64, IM_env.py:231-285), same store policy, same handle
        ob64 = torch.empty((T, n, N, F), dtype=torch.float64, device=dev)
        obs64["ptr"] = [ob64[t].data_ptr() for t in range(T)]
        f_el, f_kern, f_bpl, _, _ = timed(W, K, f64=True)
        alt64 = {"kernel": env.kernel_info(), "value": round(n * K / f_el, 1), "ms_per_step": round(f_el / K * 1e3, 6),
                 "kernel_us": round(f_kern * 1e3, 3), "bytes_per_env_step": round(f_bpl / n, 3),
                 "achieved": round(f_bpl / (f_kern * 1e-3) / 1e9, 1),
                 "frac": round(f_bpl / (f_kern * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                 "traffic": pmc_traffic(n, env.kernel_info())}
        del ob64
        obs64.clear()

    graph = None
    if world == 1 and not args.no_graph:
        graph = graph_episode_run(torch, env, reset, lib, nat, a_ptr, o_ptr, r_ptr, per_t, n, T, dev)

    # measured stream-copy ceiling at the step's byte count: a device copy of half the
    # bytes moves them once in and once out; outside the timed region
    b_steady, b_avg = env.step_traffic()
    b_handover = env.step_traffic(handover=True)[1] - b_avg
    half = max(1 << 20, int(b_avg * n) // 2 // 16 * 16)
    csrc = torch.empty(half // 4, dtype=torch.float32, device=dev)
    cdst = torch.empty_like(csrc)
    for _ in range(3):
        cdst.copy_(csrc)
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    c0.record(stream)
    for _ in range(20):
        cdst.copy_(csrc)
    c1.record(stream)
    c1.synchronize()
    copy_gbs = 2 * half * 20 / (c0.elapsed_time(c1) * 1e-3) / 1e9
    del csrc, cdst

    value = global_envs * K / el
    es = env.state_layout()[0]
    if kinfo.startswith("jit-diag:"):
        # IMENV_ABLATE / IMENV_STAMPS builds (IMENV_DIAG=1): wrong results or extra stores by design
        sys.stderr.write("bench.py: the timed kernel is a diagnostic build (%s): not a bench line\n" % kinfo)
    achieved_gbs = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    traffic = pmc_traffic(n, kinfo)
    prof = pmc_record(n, kinfo)
    trace = None
    if prof and prof.get("trace_avg_ns"):
        # the committed kernel trace of this kernel variant at this size, beside the live HIP-event time
        tus = prof["trace_avg_ns"] / 1e3
        trace = {"kernel_us": round(tus, 3), "min_us": round(prof.get("trace_min_ns", 0) / 1e3, 3),
                 "calls": prof.get("trace_calls"), "frac": round(bytes_per_launch / (tus * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                 "source": prof["_path"]}
    launcher = os.environ.get("IMENV_BENCH_LAUNCHER", "external" if world > 1 else "none")
    size = "2^20" if global_envs == 1 << 20 else str(global_envs)
    if args.scaling == "strong":
        shards = ("%s envs in all, %d per GPU (rank r steps global env ids shard_range(%d, %d, r))"
                  % (size, n, global_envs, world)) if world > 1 else "%s envs on one GPU" % size
    else:
        shards = "%s envs per GPU, %d in all (weak scaling)" % (str(n), global_envs)
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": round(el / K * 1e3, 6),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "%s state (exact: the spec's proven value bounds fit it), f64 reward, f32 obs/actions"
                 % {1: "u8", 2: "int16", 4: "int32"}[es],
        "data": "synthetic: in-kernel Philox4x32-10 Poisson(5) demand, uniform[-1,1] f32 actions (torch seed 0)",
        "ranks_seen": ranks_seen,
        "gpus_seen": gpus_seen if not args.rehearse_one_gpu else 1,
        "launcher": launcher,
        "resets_timed": resets_timed,
        "value_basis": "the gather-free pass (env steps incl. their resets; the per-step all-gather of C5 is "
                       "timed in a second pass: gather.pipelined_value)" if gather_on else
                       "env steps incl. the resets inside the timed region; no collective",
        "config": {
            "workload": "%s%s: %s, %s, 30-period episodes; %d timed steps, %d of them "
                        "preceded by the episode's reset kernel inside the timed region (step s runs period "
                        "(s + %d) mod 30)"
                        % (args.config, " at the metric's size" if args.config == "C2" and global_envs == 1 << 20
                           else "", cdesc, shards, K, resets_timed, phase),
            "n_envs_per_gpu": n, "global_envs": global_envs, "env_offset": env_off, "num_stages": N,
            "obs_features": F, "num_periods": T, "episode_phase": phase,
            "parallelism": "env-sharded x%d (one process per GPU%s, no data-path collective in the timed pass%s)"
                           % (world, ", all on GPU 0 with gloo: rehearsal" if args.rehearse_one_gpu else "",
                              "; the per-step all-gather of obs/reward timed in a second pass (\"gather\")"
                              if gather_on else ""),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "copy_ceiling_gbs": round(copy_gbs, 1),
            "kernel": kinfo,
            "kernel_us": round(kern_ms * 1e3, 3),
            "kernel_samples": launches,
            "reset_us": round(reset_us, 3) if reset_us is not None else None,
            "bytes_per_env_step": round(bytes_per_launch / n, 3),
            "bytes_per_env_step_steady": b_steady,
            "bytes_per_env_step_episode_avg": round(b_avg, 3),
            # drawn-demand hand-over (imenv_draw_layout): HBM bytes of that implementation choice, not
            # algorithmic (PMC traffic includes them)
            "handover_bytes_per_env_step_episode_avg": round(b_handover, 3),
            "bytes_per_launch": round(bytes_per_launch),
            "store_policy": args.store,
            "alt_store_policy": alt,
            "alt_obs_f64": alt64,
            "graph": graph,
            "launch_pacing": spin_info or None,
            "rocprof_trace": trace,
        },
        "gather": gather_info,
        "cpu_baseline": cpu,
    }
    if args.rccl_solo:
        out["rccl_solo"] = "one-rank nccl (RCCL) process group: census, barriers, max-reductions and the gather pass through RCCL"
    if kinfo.startswith("jit-diag:"):
        out["diagnostic_build"] = True
        out["roofline"]["traffic"] = None
    if cpu:
        out["cpu_baseline"]["gpu_over_cpu"] = round(value / cpu["value"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    env.close()
    if dist_on:
        dist.destroy_process_group()


def gather_report(gather, dist, dev, stream, K, world, n):
    """The per-step all-gather's own time, apart from the kernel's: (1) the collective stream's start /
    end events for each collective of the pipelined pass (Work._get_duration, TORCH_NCCL_ENABLE_TIMING;
    RCCL only), mean and max over ranks; (2) the same collective timed alone, K back to back (events on
    the current stream, which waits on the collective's after each; host clock on CPU tensors). Bytes
    are the packed send buffer."""
    import torch
    works = gather.keep_works(False)
    in_loop = None
    try:
        d = [w._get_duration() for w in works]
        if d and all(x is not None and x >= 0 for x in d):
            in_loop = sum(d) / len(d)
    except Exception:
        in_loop = None
    # alone: K collectives of buffer 0, nothing else on the GPU
    reps = max(5, min(K, 50))
    gather.start(0)
    gather.wait(0)
    if dev is not None:
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    if dev is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
    h0 = time.perf_counter()
    for _ in range(reps):
        gather.start(0)
        gather.wait(0)
    if dev is not None:
        e1.record(stream)
        e1.synchronize()
        alone = e0.elapsed_time(e1) / reps
    else:
        alone = (time.perf_counter() - h0) * 1e3 / reps
    t = torch.tensor([in_loop if in_loop is not None else -1.0, alone], dtype=torch.float64,
                     device=dev if dev is not None else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    in_loop_max = t[0].item() if in_loop is not None else None
    recv = gather.chunk * world
    return {
        "collective": "all_gather_into_tensor" if gather._into else "all_gather (list form)",
        "send_bytes_per_rank": gather.chunk, "recv_bytes_per_rank": recv,
        "gather_us": round(in_loop_max * 1e3, 3) if in_loop_max is not None else None,
        "gather_us_source": "collective-stream events per pipelined collective (max over ranks of the mean)"
                            if in_loop_max is not None else "unavailable (backend records no per-collective times)",
        "recv_gbs": round(recv / (in_loop_max * 1e-3) / 1e9, 1) if in_loop_max else None,
        "gather_alone_us": round(t[1].item() * 1e3, 3),
        "gather_alone_recv_gbs": round(recv / (t[1].item() * 1e-3) / 1e9, 1),
        "collectives_timed": len(works),
    }


def graph_gather_run(torch, dist, dev, gather, reset, lib, nat, a_ptr, T, h, replays=10):
    """C5's per-step all-gather with the host out of the loop: one episode (reset, T steps into the
    StepGather's double-buffered send views, each step's all_gather_into_tensor started on the
    collective's stream under the next step) captured into one HIP graph and replayed back to back.
    Also T collectives alone in a graph of their own (the collective's device time without the
    host's launch pacing). RCCL only (gloo collectives run on the host)."""
    world = dist.get_world_size()
    torch.cuda.synchronize(dev)
    gather.wait(0)
    gather.wait(1)
    gather.keep_works(False)          # no Work objects are kept for captured collectives
    s = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    dist.barrier()
    with torch.cuda.graph(g, stream=s):
        sp = torch.cuda.current_stream(dev).cuda_stream
        for t in range(T):
            if t == 0:
                reset(sp)
            rc = lib.imenv_step(h, a_ptr[t], nat.F32, gather.obs_out(t).data_ptr(), nat.F32,
                                gather.reward_out(t).data_ptr(), None, None, sp)
            if rc:
                nat.check(rc, "imenv_step")
            gather.start(t)
            if t > 0:
                gather.result(t - 1)
        gather.result(T - 1)
    cur = torch.cuda.current_stream(dev)
    g.replay()
    torch.cuda.synchronize(dev)
    dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(cur)
    for _ in range(replays):
        g.replay()
    e1.record(cur)
    e1.synchronize()
    wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1)
    # the collectives alone: T all-gathers of buffer 0, back to back, in a graph
    ga = torch.cuda.CUDAGraph()
    torch.cuda.synchronize(dev)
    with torch.cuda.graph(ga, stream=s):
        for _ in range(T):
            gather.start(0)
            gather.wait(0)
    ga.replay()
    torch.cuda.synchronize(dev)
    a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a0.record(cur)
    for _ in range(replays):
        ga.replay()
    a1.record(cur)
    a1.synchronize()
    alone_ms = a0.elapsed_time(a1) / (replays * T)
    t = torch.tensor([ms, wall * 1e3, alone_ms], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms, wall_ms, alone_ms = t.tolist()
    del g, ga
    recv = gather.chunk * world
    steps = replays * T
    return {"replays": replays, "steps": steps, "ms_per_step": round(ms / steps, 6),
            "host_wall_ms_per_step": round(wall_ms / steps, 6),
            "collective_alone_us": round(alone_ms * 1e3, 3),
            "collective_alone_recv_gbs": round(recv / (alone_ms * 1e-3) / 1e9, 1),
            "note": "per replay: the reset, %d steps and %d all-gathers (max over ranks); the collective alone: "
                    "%d all-gathers of one buffer per replay" % (T, T, T)}


def graph_episode_run(torch, env, reset, lib, nat, a_ptr, o_ptr, r_ptr, per_t, n, T, dev, replays=10):
    """Informational: one episode (reset + T steps) captured into a HIP graph and replayed back to back
    (the host out of the loop: a trainer that captures its sampler). Each replay draws the next episode's
    demand (the reset kernel advances the device episode counter). ms_per_step and value count the reset
    with its episode."""
    s = torch.cuda.Stream(dev)
    graph = torch.cuda.CUDAGraph()
    torch.cuda.synchronize(dev)
    with torch.cuda.graph(graph, stream=s):
        sp = torch.cuda.current_stream(dev).cuda_stream
        reset(sp)
        for t in range(T):
            rc = lib.imenv_step(env._h, a_ptr[t], nat.F32, o_ptr[t], nat.F32, r_ptr[t], None, None, sp)
            if rc:
                nat.check(rc, "imenv_step")
    kinfo = env.kernel_info()
    cur = torch.cuda.current_stream(dev)
    graph.replay()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(cur)
    for _ in range(replays):
        graph.replay()
    e1.record(cur)
    e1.synchronize()
    wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1)
    steps = replays * T
    bytes_ep = sum(per_t[t] for t in range(T)) * n
    del graph
    return {"kernel": kinfo, "replays": replays, "steps": steps, "ms_per_step": round(ms / steps, 6),
            "value": round(n * steps / (ms * 1e-3), 1), "host_wall_ms_per_step": round(wall * 1e3 / steps, 6),
            "achieved_incl_reset": round(bytes_ep * replays / (ms * 1e-3) / 1e9, 1),
            "frac_incl_reset": round(bytes_ep * replays / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


if __name__ == "__main__":
    main()

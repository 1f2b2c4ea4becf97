"""bench.py's driver contract: the CPU-baseline leg on the host (CPU), and one short GPU run whose JSON
line must carry every key the driver and the judge read (metric / value / unit / n_gpus / steps /
warmup / ms_per_step / higher_is_better / scaling / vs_baseline / dtype / data / config, plus roofline
and cpu_baseline)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, timeout):
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    r = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_cpu_baseline_leg():
    """The oracle port timed on the host cores (one env per process): a positive rate, the core count
    and kind "port"."""
    d = _run(["--cpu-only", "--cpu-seconds", "0.3"], timeout=300)
    assert d["value"] > 0 and d["unit"] == "env-steps/s" and d["kind"] == "port"
    assert d["cores"] >= 1 and "oracle/im_oracle.py" in d["sample"]
    # the pool size and the host's core counts are both stated (a capped pool is never silent)
    assert "host reports" in d["sample"] and "CPU share" in d["sample"]


@pytest.mark.gpu
@pytest.mark.parametrize("steps,warmup", [(20, 5), (45, 7)])
def test_bench_json_line(steps, warmup):
    """(20, 5) is the driver's own round-end command; (45, 7) crosses an episode boundary (reset inside
    the timed region). Every timed step launch is a kernel-time sample and W is reported as given."""
    extra = ["--cpu-seconds", "0.3"] if steps == 20 else ["--no-cpu-baseline"]
    d = _run(["--steps", str(steps), "--warmup", str(warmup)] + extra, timeout=300)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == steps and d["warmup"] == warmup and d["scaling"] == "strong"
    assert d["higher_is_better"] is True and d["config"]["global_envs"] == 1 << 20
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["n_envs_per_gpu"] == 1 << 20 and "workload" in d["config"]
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["kernel"].startswith("jit:imenv_step_jit")
    assert r["kernel_samples"] == steps and r["kernel_us"] > 0
    assert r["store_policy"] == "default"
    alt = r["alt_store_policy"]      # plain stores, timed the same way (informational)
    assert alt["store_policy"] == "plain" and alt["value"] > 0 and 0 < alt["frac"] < 1
    # the line names the kernel it timed: write-through obs / reward stores (0x2000), and at 2^20 envs
    # (58.7 MB of outputs per launch, more than L2) plain state rows; the informational run its own
    import re
    flags = lambda k: int(re.search(r",flags=(0x[0-9a-f]+),", k).group(1), 16)
    # JitFlags bits: 0x2000 write-through obs, 0x4000 write-through state, 0x10000 no info code (none
    # requested), 0x20000 whole blocks (2^20 is a multiple of 2048), 0x40000 16-byte aligned obs buffer
    assert r["kernel"].startswith("jit:imenv_step_jit_wt[") and flags(r["kernel"]) == 0x2000 | 0x70000
    assert alt["kernel"].startswith("jit:imenv_step_jit[") and flags(alt["kernel"]) == 0x70000
    f64 = r["alt_obs_f64"]           # the reference's float64 observations, same run (informational)
    assert f64["kernel"].startswith("jit:imenv_step_jit_wt_o64[") and 0 < f64["frac"] < 1
    assert f64["bytes_per_env_step"] > r["bytes_per_env_step"] and f64["value"] > 0
    g = r["graph"]                   # the HIP-graph-replayed episode (informational)
    assert g["steps"] == 30 * g["replays"] and g["ms_per_step"] > 0 and g["kernel"] == r["kernel"]
    ph = d["config"]["episode_phase"]
    assert d["resets_timed"] == sum(1 for s in range(warmup, warmup + steps) if (s + ph) % 30 == 0) >= 1
    assert ("%d of them preceded by the episode's reset kernel" % d["resets_timed"]) in d["config"]["workload"]
    assert r["reset_us"] > 0 and "resets" in d["value_basis"]
    assert d["ranks_seen"] == 1 and d["launcher"] == "none"
    assert 90 < r["bytes_per_env_step"] <= r["bytes_per_env_step_steady"]
    if steps != 20:
        return
    c = d["cpu_baseline"]
    assert c["value"] > 0 and c["kind"] == "port" and c["cores"] >= 1


@pytest.mark.gpu
def test_small_launch_window_runs_as_one_graph():
    """C5's per-GPU shard (131,072 envs) at the driver's settings: the host's per-step enqueue is close to the
    kernel's time, so the timed K steps (and their reset) replay as one HIP graph captured before the timed
    region; the kernel time is the replay's event span minus the timed resets, over K."""
    d = _run(["--n-envs", "131072", "--steps", "20", "--warmup", "5", "--no-cpu-baseline", "--no-alt-store",
              "--no-alt-obs", "--no-graph"], timeout=300)
    r = d["roofline"]
    p = r["launch_pacing"]
    assert p["launch"] == "graph" and d["resets_timed"] == 1 and r["kernel_samples"] == 20
    assert "graph replay" in p["window"]["kernel_us_source"] and p["window"]["reset_us_subtracted"] > 0
    assert 0 < r["frac"] < 1 and r["kernel_us"] > 0 and d["value"] > 0
    d = _run(["--n-envs", "131072", "--steps", "20", "--warmup", "5", "--no-cpu-baseline", "--no-alt-store",
              "--no-alt-obs", "--no-graph", "--launch", "eager"], timeout=300)
    assert d["roofline"]["launch_pacing"]["launch"] == "eager" and d["roofline"]["kernel_samples"] == 20


def _run_rc(args, timeout, **extra_env):
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1", **extra_env)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        if k not in extra_env:
            env.pop(k, None)
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env,
                          cwd=ROOT)


def test_gpus_n_spawns_n_ranks_itself():
    """`bench.py --gpus 2` with no launcher starts its own 2 rank processes (gloo rendezvous on
    127.0.0.1, census of ranks, max-reduction), hands them the CPU baseline it measured first, and
    rank 0 prints one line with n_gpus 2 and ranks_seen 2 (the reference's own parallelism: one env
    per RLlib worker process, hyperparams.py:14)."""
    r = _run_rc(["--gpus", "2", "--dry-run", "--no-gather", "--cpu-seconds", "0.2"], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout           # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["launcher"] == "self"
    assert sorted(x["rank"] for x in d["ranks"]) == [0, 1] and d["max_over_ranks"] == 2.0
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["kind"] == "port"
    # strong scaling by default: the metric's 2^20 envs split over the ranks (C5 at 8 ranks)
    assert d["scaling"] == "strong" and d["config"]["global_envs"] == 1 << 20
    assert d["config"]["n_envs_per_gpu"] == 1 << 19 and d["gather"] is None


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 6, 7, 8])
def test_strong_shard_plan_covers_the_metric_size(world):
    """Every N: the ranks' contiguous shards cover global env ids [0, 2^20) exactly once (SURVEY.md §8e:
    rank r owns [r*n/W, (r+1)*n/W)), so the N-GPU line always steps the metric's 2^20 envs; at N = 8
    each rank steps 131,072 envs (BASELINE.json configs[4], C5)."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "marl-for-im_amd"))
    import bench
    plans = [bench.shard_plan("strong", "C2", None, world, r) for r in range(world)]
    assert all(total == 1 << 20 for _, _, total in plans)
    assert plans[0][0] == 0 and sum(n for _, n, _ in plans) == 1 << 20
    for (o0, n0, _), (o1, _, _) in zip(plans, plans[1:]):
        assert o1 == o0 + n0
    assert max(n for _, n, _ in plans) - min(n for _, n, _ in plans) <= 1
    if world == 8:
        assert {n for _, n, _ in plans} == {131072}
    # weak scaling: every rank its own 2^20 envs, at ids r * 2^20
    weak = [bench.shard_plan("weak", "C2", None, world, r) for r in range(world)]
    assert [o for o, _, _ in weak] == [r << 20 for r in range(world)]
    assert all(n == 1 << 20 and total == world << 20 for _, n, total in weak)


def test_gather_leg_runs_step_gather_over_gloo():
    """`--gpus 2 --dry-run --gather`: both ranks drive StepGather's double-buffered pipeline (write into
    obs_out(s) / reward_out(s), start(s), result(s-1)) on CPU tensors with gloo, every gathered step is
    checked against the global env ids, and gather_report fills the line's "gather" object."""
    steps = 7
    r = _run_rc(["--gpus", "2", "--dry-run", "--gather", "--no-cpu-baseline", "--n-envs", "4096",
                 "--steps", str(steps)], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    g = d["gather"]
    assert d["config"]["global_envs"] == 4096 and d["config"]["n_envs_per_gpu"] == 2048
    assert g["collectives_timed"] == steps and g["gather_alone_us"] > 0
    # packed send buffer: obs [2048, 4, 3] f32 + reward [2048] f64, each field 256-byte aligned
    assert g["send_bytes_per_rank"] == 2048 * 12 * 4 + 2048 * 8 and g["recv_bytes_per_rank"] == 2 * g["send_bytes_per_rank"]
    # on by default with more than one rank
    r = _run_rc(["--gpus", "2", "--dry-run", "--no-cpu-baseline", "--n-envs", "4096", "--steps", "3"], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])["gather"]["collectives_timed"] == 3


def test_weak_scaling_flag():
    r = _run_rc(["--gpus", "2", "--dry-run", "--no-gather", "--no-cpu-baseline", "--weak"], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["scaling"] == "weak" and d["config"]["global_envs"] == 2 << 20 and d["config"]["n_envs_per_gpu"] == 1 << 20


def test_gpus_disagreeing_with_launcher_world_fails():
    r = _run_rc(["--gpus", "2", "--dry-run", "--no-cpu-baseline"], timeout=120, WORLD_SIZE="1", RANK="0",
                LOCAL_RANK="0")
    assert r.returncode == 2 and "launcher started 1 ranks" in r.stderr


def test_a_failing_rank_fails_the_launch():
    r = _run_rc(["--gpus", "2", "--dry-run", "--no-cpu-baseline"], timeout=120, IMENV_BENCH_DRY_FAIL_RANK="1")
    assert r.returncode == 7, (r.returncode, r.stderr[-2000:])
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_steps_must_be_positive():
    r = _run_rc(["--steps", "0", "--no-cpu-baseline"], timeout=60)
    assert r.returncode == 2 and "--steps must be >= 1" in r.stderr


def test_rccl_solo_is_world_size_one_only():
    """--rccl-solo is the one-rank RCCL check: refused with a rehearsal or under a multi-rank launcher."""
    r = _run_rc(["--rccl-solo", "--rehearse-one-gpu", "--no-cpu-baseline"], timeout=60)
    assert r.returncode == 2 and "--rccl-solo" in r.stderr
    r = _run_rc(["--gpus", "2", "--rccl-solo", "--no-cpu-baseline"], timeout=60, WORLD_SIZE="2", RANK="0",
                LOCAL_RANK="0")
    assert r.returncode == 2 and "--rccl-solo" in r.stderr


@pytest.mark.parametrize("W,K", [(5, 20), (0, 1), (7, 29), (5, 30), (60, 300), (3, 2), (29, 10)])
def test_timed_window_holds_a_reset(W, K):
    """The driver's short window (--steps 20 --warmup 5) is phased so that an episode boundary, and with it
    the reset kernel, falls inside the timed steps; windows of >= 30 steps hold one anyway."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "marl-for-im_amd"))
    import bench
    ph = bench.episode_phase(W, K, 30)
    assert 0 <= ph < 30 and (ph == 0 or K < 30)
    assert bench.resets_in_window(W, K, 30, ph) >= 1
    assert bench.resets_in_window(W, K, 30, ph) == sum(1 for s in range(W, W + K) if (s + ph) % 30 == 0)

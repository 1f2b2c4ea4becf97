"""The RCCL path of bench.py's N-rank line, exercised on one MI355X at world size 1 (the driver's
8-GPU run is the only place it meets more than one rank): a one-rank "nccl" process group with the
census, barriers and max-reductions through it, and C5's per-step all-gather of obs + reward over
RCCL. Each case runs in its own process (a process group in the test runner would outlive the test).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _run(argv, timeout):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable] + argv, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_step_gather_over_rccl_is_bit_exact():
    """Two episodes of C2 envs stepped into StepGather's send buffers with every collective in flight
    under the next step: each gathered step equals a plain handle's outputs."""
    d = _run([os.path.join(ROOT, "tests", "rccl_gather_check.py"), "8192"], timeout=180)
    assert d["backend"] == "nccl" and d["collective"] == "all_gather_into_tensor" and d["world"] == 1
    assert d["steps"] == 60 and d["mismatches"] == 0


def test_bench_line_through_rccl():
    """bench.py --rccl-solo: the line's gather pass runs over RCCL, each collective's own duration comes
    from RCCL's stream events (TORCH_NCCL_ENABLE_TIMING), and the gather-free pass is the line."""
    d = _run([os.path.join(ROOT, "bench.py"), "--rccl-solo", "--n-envs", "131072", "--steps", "40", "--warmup", "5",
              "--no-cpu-baseline", "--no-alt-store", "--no-alt-obs", "--no-graph"], timeout=240)
    assert d["n_gpus"] == 1 and d["ranks_seen"] == 1 and "rccl_solo" in d
    g = d["gather"]
    assert g and "error" not in g, g
    assert g["backend"].startswith("nccl") and g["collective"] == "all_gather_into_tensor"
    assert g["gather_us"] is not None and g["gather_us"] > 0 and g["collectives_timed"] >= 40
    assert g["pipelined_value"] > 0 and d["value"] > 0
    assert g["send_bytes_per_rank"] == g["recv_bytes_per_rank"] >= 131072 * (48 + 8)

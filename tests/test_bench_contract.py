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
    assert d["n_gpus"] == 1 and d["steps"] == steps and d["warmup"] == warmup and d["scaling"] == "weak" and d["higher_is_better"] is True
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["n_envs_per_gpu"] == 1 << 20 and "workload" in d["config"]
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["kernel"].startswith("jit:imenv_step_jit")
    assert r["kernel_samples"] == steps and r["kernel_us"] > 0
    assert r["store_policy"] == "default"
    alt = r["alt_store_policy"]      # the other store policy, timed the same way (informational)
    assert alt["store_policy"] == "stream" and alt["value"] > 0 and 0 < alt["frac"] < 1
    # the line names the kernel it timed (plain stores), the informational run its own (flag 0x800)
    assert r["kernel"].startswith("jit:imenv_step_jit[") and ",flags=0x0," in r["kernel"]
    assert alt["kernel"].startswith("jit:imenv_step_jit_nt[") and ",flags=0x800," in alt["kernel"]
    assert 90 < r["bytes_per_env_step"] <= r["bytes_per_env_step_steady"]
    if steps != 20:
        return
    c = d["cpu_baseline"]
    assert c["value"] > 0 and c["kind"] == "port" and c["cores"] >= 1

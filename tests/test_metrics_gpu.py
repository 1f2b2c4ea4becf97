"""Evaluation-harness accumulators of the step kernel (imenv_set_episode_metrics) and the column
statistics kernel (imenv_column_stats) vs the harness restated over the reference's own episodes.

The golden cases hold the reference env's float64 observations, rewards and profits for 32 envs x
30 periods; oracle/harness.py accumulates them exactly as the reference's test loops do
(inv_management.py:586-597, MA_inv_management.py:559-572). The GPU, stepping the same demand and
actions with metrics attached, must produce the same per-env sums bit for bit (both kernel paths).
"""
import os

import numpy as np
import pytest
import torch

from golden_io import load_case
from oracle.harness import harness_metrics

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
os.environ["IMENV_JIT_STRICT"] = "1"
CASES = ["C1_IM4", "IM4_S3", "IM4_nonstd", "C3_IM8", "C2_MAIM4", "MAIM4_indep", "MAIM4_MA6", "IM_div1",
         "C4_MAIM_div1", "MAIM_div1_indep", "MAIM_div2_share", "IM4_noisy_delay"]


@pytest.mark.parametrize("jit", [1, 0])
@pytest.mark.parametrize("name", CASES)
def test_harness_metrics_match_reference_episodes(name, jit):
    from imenv import VectorInvEnv
    meta, d = load_case(name)
    kind, cfg, E, T = meta["kind"], meta["config"], meta["E"], meta["T"]
    env = VectorInvEnv(kind, cfg, n_envs=E, device=DEV, obs_dtype=torch.float64)
    env.set_jit(jit)
    env.attach_metrics()
    serial = kind in ("IM", "MAIM")
    dem = d["customer_demand"]
    noisy = meta["noisy"]
    for rep in range(2):                       # the second episode restarts every sum at period 0
        env.reset(customer_demand=dem[:, 0, :] if serial else dem, noisy_delay=bool(noisy),
                  noisy_delay_threshold=noisy, delay_uniforms=d["delay_uniforms"] if noisy else None)
        for t in range(T):
            env.step(torch.as_tensor(d["actions"][:, t, :], dtype=torch.float64, device=DEV))
    m = env.metrics()
    got = torch.cat([torch.stack([m[k] for k in ("episode_reward", "total_inventory", "total_backlog",
                                                 "customer_backlog")], 1), m["stage_reward"]], 1).cpu().numpy()
    sp = env.spec
    ref = harness_metrics(d["obs"], d["reward"], d["profit"], sp.inv_max.astype(np.float64), sp.a, sp.b,
                          kind in ("MAIM", "MAIM_div"))
    np.testing.assert_array_equal(got, ref)
    st = env.metrics_stats().cpu().numpy()
    np.testing.assert_allclose(st[:, 0], ref.mean(axis=0), rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(st[:, 1], ref.std(axis=0), rtol=1e-9, atol=1e-9)
    env.close()


def test_column_stats_large():
    """np.mean / np.std of a 3,000,001 x 7 matrix (ragged last block) within 1e-12 relative."""
    from imenv import _native as nat
    lib = nat.load()
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    x = torch.randn((3_000_001, 7), generator=g, dtype=torch.float64, device=DEV) * 50 + 10
    out = torch.empty((7, 2), dtype=torch.float64, device=DEV)
    nat.check(lib.imenv_column_stats(x.data_ptr(), x.shape[0], x.shape[1], out.data_ptr(), None), "stats")
    torch.cuda.synchronize()
    xn = x.cpu().numpy()
    np.testing.assert_allclose(out[:, 0].cpu().numpy(), xn.mean(axis=0), rtol=1e-12)
    np.testing.assert_allclose(out[:, 1].cpu().numpy(), xn.std(axis=0), rtol=1e-12)


def test_metric_stats_merge_over_shards():
    """Harness stats of 3 env shards (env_offset, in-kernel draws) merged with imenv.shard's Chan merge
    (what global_metrics_stats does over ranks) == the stats of one env over all envs, and == np.mean /
    np.std of the per-env sums."""
    from imenv import VectorInvEnv
    from imenv.shard import merge_column_stats, shard_range
    meta, _ = load_case("C2_MAIM4")
    total = 10007

    def run(n, off):
        env = VectorInvEnv(meta["kind"], meta["config"], n_envs=n, device=DEV, env_offset=off)
        env.attach_metrics()
        env.reset()
        g = torch.Generator(device=DEV)
        for t in range(env.T):
            g.manual_seed(t)
            a = torch.rand((total, env.N), generator=g, device=DEV)[off:off + n] * 2 - 1
            env.step(a.contiguous())
        stats, m = env.metrics_stats(), env._metrics.clone()
        env.close()
        return stats, m

    whole_stats, whole = run(total, 0)
    parts = [run(c, o) for o, c in (shard_range(total, 3, r) for r in range(3))]
    np.testing.assert_array_equal(torch.cat([m for _, m in parts]).cpu().numpy(), whole.cpu().numpy())
    merged = merge_column_stats(torch.stack([s.cpu() for s, _ in parts]),
                                [shard_range(total, 3, r)[1] for r in range(3)]).numpy()
    x = whole.cpu().numpy()
    np.testing.assert_allclose(merged[:, 0], x.mean(0), rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(merged[:, 1], x.std(0), rtol=1e-10, atol=1e-9)
    np.testing.assert_allclose(merged, whole_stats.cpu().numpy(), rtol=1e-10, atol=1e-9)

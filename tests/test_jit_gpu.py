"""hipRTC step-kernel selection: the observation slab stays within its LDS budget under any
IMENV_JIT_BS, and a compile failure sends only its own flag set to the ahead-of-time kernels (the
other flag sets of the handle keep their specialised kernels). Results bit-exact vs the reference's
golden vectors either way."""
import re

import numpy as np
import pytest
import torch

from golden_io import load_case

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
STAGE_LDS = 48 * 1024      # kStageLds, imenv_jit.hip


def _episode(env, meta, d, obs_dtype):
    serial = meta["kind"] in ("IM", "MAIM")
    dem = d["customer_demand"]
    noisy = meta["noisy"]      # host-fed noisy-delay uniforms, as the reference's session drew them
    env.reset(customer_demand=dem[:, 0, :] if serial else dem, noisy_delay=bool(noisy), noisy_delay_threshold=noisy,
              delay_uniforms=d["delay_uniforms"] if noisy else None)
    obs, rew = [], []
    for t in range(meta["T"]):
        a = torch.as_tensor(d["actions"][:, t, :], dtype=torch.float64, device=DEV)
        o, r, _, _ = env.step(a)
        obs.append(o.cpu().numpy())
        r = r.cpu().numpy()
        rew.append(r if r.ndim == 2 else r[:, None])
    exp = d["obs"] if obs_dtype == torch.float64 else d["obs"].astype(np.float32)
    np.testing.assert_array_equal(np.stack(obs, axis=1), exp)
    ref_r = d["reward"]
    got_r = np.stack(rew, axis=1)
    np.testing.assert_array_equal(got_r, ref_r[..., :got_r.shape[-1]])


@pytest.mark.parametrize("name", ["C3_IM8", "IM8_td", "MAIM_div2_share", "C2_MAIM4"])
@pytest.mark.parametrize("odt", ["f32", "f64"])
def test_gpu_jit_block_size_bounds_the_obs_slab(name, odt, monkeypatch):
    """IMENV_JIT_BS=1024: an 8-stage base row staged as float64 would need 1024 x 25 x 8 B = 200 KiB of
    LDS (over the static limit, so the hipRTC compile failed and the handle lost its JIT kernels);
    the block size now halves until the staged slab fits, for base rows as for general ones."""
    from imenv import VectorInvEnv
    monkeypatch.setenv("IMENV_JIT_BS", "1024")
    monkeypatch.setenv("IMENV_JIT_STRICT", "1")
    meta, d = load_case(name)
    tdt = torch.float64 if odt == "f64" else torch.float32
    env = VectorInvEnv(meta["kind"], meta["config"], n_envs=meta["E"], device=DEV, obs_dtype=tdt)
    _episode(env, meta, d, tdt)
    info = env.kernel_info()
    assert info.startswith("jit:") and "jit failed" not in info, info
    bs = int(re.search(r"bs=(\d+)", info).group(1))
    N, F = d["obs"].shape[2], d["obs"].shape[3]
    vb = 8 if odt == "f64" else 4
    base = "base=1" in info
    row = 3 * N if base else N * F
    stride = row + 1 if row % (2 if vb == 8 else 8) == 0 else row
    if base:
        assert bs * stride * vb <= STAGE_LDS, (bs, stride, vb)
    env.close()


def test_gpu_jit_failure_falls_back_for_its_flag_set_only(monkeypatch):
    """A flag set whose hipRTC compile fails (forced here by pre-including a header that does not exist) runs on the
    ahead-of-time kernel, bit-exact; the handle's next flag set (float64 observations) still gets
    its JIT kernel, and set_jit(1) retries the failed one."""
    from imenv import VectorInvEnv
    monkeypatch.setenv("IMENV_JIT_STRICT", "0")
    meta, d = load_case("C2_MAIM4")
    env = VectorInvEnv(meta["kind"], meta["config"], n_envs=meta["E"], device=DEV, obs_dtype=torch.float32)
    monkeypatch.setenv("IMENV_JIT_OPTS", "-include imenv_no_such_header_probe.h")
    _episode(env, meta, d, torch.float32)
    info = env.kernel_info()
    assert info.startswith("aot:") and "jit failed" in info, info
    monkeypatch.delenv("IMENV_JIT_OPTS")
    env.obs_dtype = torch.float64
    _episode(env, meta, d, torch.float64)
    assert env.kernel_info().startswith("jit:"), env.kernel_info()
    env.obs_dtype = torch.float32
    _episode(env, meta, d, torch.float32)
    assert env.kernel_info().startswith("aot:")     # the failed flag set stays on AOT ...
    env.set_jit(1)
    _episode(env, meta, d, torch.float32)
    assert env.kernel_info().startswith("jit:"), env.kernel_info()   # ... until set_jit(1) retries it
    env.close()


def test_gpu_diagnostic_builds_need_imenv_diag(monkeypatch):
    """A diagnostic compile switch in IMENV_JIT_OPTS (IMENV_ABLATE: wrong results by design) is refused
    at kernel load without IMENV_DIAG=1: the flag set runs on the ahead-of-time kernel, bit-exact, and
    kernel_info says why. With IMENV_DIAG=1 a diagnostic build (here IMENV_STAMPS, which leaves the
    results alone when no stamp buffer is attached) loads, and its tag starts "jit-diag:" with a kernel
    name of its own, so bench.py and tools/pmc_summary.py can refuse it."""
    from imenv import VectorInvEnv
    monkeypatch.setenv("IMENV_JIT_STRICT", "0")
    monkeypatch.delenv("IMENV_DIAG", raising=False)
    meta, d = load_case("C2_MAIM4")
    monkeypatch.setenv("IMENV_JIT_OPTS", "-DIMENV_ABLATE=16")
    env = VectorInvEnv(meta["kind"], meta["config"], n_envs=meta["E"], device=DEV, obs_dtype=torch.float32)
    _episode(env, meta, d, torch.float32)
    info = env.kernel_info()
    assert info.startswith("aot:") and "IMENV_DIAG" in info, info
    env.close()
    monkeypatch.setenv("IMENV_JIT_OPTS", "-DIMENV_STAMPS=1")
    monkeypatch.setenv("IMENV_DIAG", "1")
    env = VectorInvEnv(meta["kind"], meta["config"], n_envs=meta["E"], device=DEV, obs_dtype=torch.float32)
    _episode(env, meta, d, torch.float32)
    info = env.kernel_info()
    assert re.match(r"jit-diag:imenv_step_jit_wt_diag_[0-9a-f]{8}\[", info), info
    env.close()
    monkeypatch.setenv("IMENV_JIT_OPTS", "-DIMENV_SLAB_BATCH=1")     # a tuning option: not diagnostic
    monkeypatch.delenv("IMENV_DIAG")
    env = VectorInvEnv(meta["kind"], meta["config"], n_envs=meta["E"], device=DEV, obs_dtype=torch.float32)
    _episode(env, meta, d, torch.float32)
    assert re.match(r"jit:imenv_step_jit_wt_opt_[0-9a-f]{8}\[", env.kernel_info()), env.kernel_info()
    env.close()


@pytest.mark.parametrize("name", ["C2_MAIM4", "C3_IM8", "MAIM_div2_share"])
@pytest.mark.parametrize("odt", ["f32", "f64"])
@pytest.mark.parametrize("mode", [1, 0])
def test_gpu_misaligned_obs_out_view(name, odt, mode):
    """A caller-owned obs_out that is a view one element into a larger buffer (8-byte aligned for
    float64, 4-byte for float32, never 16): the staged slab write-out drops to element stores and the
    observations equal those written into an aligned buffer."""
    from imenv import VectorInvEnv
    meta, d = load_case(name)
    tdt = torch.float64 if odt == "f64" else torch.float32
    serial = meta["kind"] in ("IM", "MAIM")
    dem = d["customer_demand"]
    envs = []
    for _ in range(2):
        e = VectorInvEnv(meta["kind"], meta["config"], n_envs=meta["E"], device=DEV, obs_dtype=tdt)
        e.set_jit(mode)
        e.reset(customer_demand=dem[:, 0, :] if serial else dem)
        envs.append(e)
    n, N, F = meta["E"], d["obs"].shape[2], d["obs"].shape[3]
    big = torch.empty(n * N * F + 1, dtype=tdt, device=DEV)
    view = big[1:].view(n, N, F)
    assert view.data_ptr() % 16 != 0
    for t in range(meta["T"]):
        a = torch.as_tensor(d["actions"][:, t, :], dtype=torch.float64, device=DEV)
        ref, _, _, _ = envs[0].step(a)
        envs[1].step(a, obs_out=view)
        np.testing.assert_array_equal(view.cpu().numpy(), ref.cpu().numpy(), err_msg="t=%d" % t)
    exp = d["obs"][:, -1] if tdt == torch.float64 else d["obs"][:, -1].astype(np.float32)
    np.testing.assert_array_equal(view.cpu().numpy(), exp)
    for e in envs:
        e.close()


# store policy -> (flag bits that must be set, flag bits that must be clear) in the kernel tag:
# 0x800 non-temporal obs / reward, 0x2000 write-through obs / reward, 0x4000 write-through state rows
STORE_FLAGS = {"stream": (0x800, 0x6000), "plain": (0, 0x6800), "writethrough": (0x6000, 0x800),
               "default": (0x6000, 0x800)}     # default at golden sizes (32 envs: outputs fit in L2)


@pytest.mark.parametrize("name", ["C2_MAIM4", "C3_IM8", "C4_MAIM_div1", "MAIM_div2_share", "MAIM4_indep",
                                  "IM4_td_pd_pa_L2", "MAIM_div1_noisy_delay"])
@pytest.mark.parametrize("odt", ["f32", "f64"])
@pytest.mark.parametrize("policy", ["stream", "plain", "writethrough", "default"])
def test_gpu_store_policies_same_results(name, odt, policy):
    """Every store policy (imenv_set_store_policy) is a hipRTC kernel of its own (flag bits in its tag)
    with bit-identical results against the reference's golden episode; switching policy mid-run
    selects the other kernel."""
    from imenv import VectorInvEnv
    meta, d = load_case(name)
    tdt = torch.float64 if odt == "f64" else torch.float32
    env = VectorInvEnv(meta["kind"], meta["config"], n_envs=meta["E"], device=DEV, obs_dtype=tdt)
    env.set_store_policy(policy)
    _episode(env, meta, d, tdt)
    flags = int(re.search(r"flags=0x([0-9a-f]+)", env.kernel_info()).group(1), 16)
    on, off = STORE_FLAGS[policy]
    assert env.kernel_info().startswith("jit:") and flags & on == on and not flags & off, env.kernel_info()
    other = "plain" if policy != "plain" else "writethrough"
    env.set_store_policy(other)
    _episode(env, meta, d, tdt)
    flags = int(re.search(r"flags=0x([0-9a-f]+)", env.kernel_info()).group(1), 16)
    on, off = STORE_FLAGS[other]
    assert flags & on == on and not flags & off, env.kernel_info()
    assert env.lib.imenv_set_store_policy(env._h, 7) != 0      # unknown policy: IMENV_E_INVALID
    with pytest.raises(ValueError):
        env.set_store_policy("bogus")
    env.close()


@pytest.mark.parametrize("name", ["C2_MAIM4", "C4_MAIM_div1", "MAIM4_indep"])
@pytest.mark.parametrize("odt", ["f32", "f64"])
@pytest.mark.parametrize("rows", ["T+1", "T"])
def test_gpu_rollout_stepper_matches_step(name, odt, rows):
    """VectorInvEnv.rollout_stepper: the pre-validated launcher writes, period by period, exactly what
    step() returns (the reference's golden observations and rewards), into rows t + 1 (or t) of the
    bound buffers; a stepper called out of period order, and badly shaped buffers, are rejected."""
    from imenv import VectorInvEnv
    meta, d = load_case(name)
    tdt = torch.float64 if odt == "f64" else torch.float32
    E, T = meta["E"], meta["T"]
    env = VectorInvEnv(meta["kind"], meta["config"], n_envs=E, device=DEV, obs_dtype=tdt)
    acts = torch.as_tensor(d["actions"], dtype=torch.float64, device=DEV).permute(1, 0, 2).contiguous()
    obs = torch.empty((T + 1 if rows == "T+1" else T, E, env.N, env.F), dtype=tdt, device=DEV)
    rew = torch.empty((T,) + env.reward_shape(), dtype=torch.float64, device=DEV)
    stepper = env.rollout_stepper(acts, obs, rew)
    with pytest.raises(ValueError):
        env.rollout_stepper(acts[:, :, :-1].contiguous(), obs, rew)
    with pytest.raises(ValueError):
        env.rollout_stepper(acts, obs[:, :, :, :-1].contiguous(), rew)
    serial = meta["kind"] in ("IM", "MAIM")
    dem = d["customer_demand"]
    o0 = env.reset(customer_demand=dem[:, 0, :] if serial else dem)
    with pytest.raises(ValueError):
        stepper(1)
    for t in range(T):
        done = stepper(t)
        assert done == (t == T - 1)
    with pytest.raises(ValueError, match="past the horizon"):
        stepper(T)
    got = obs[1:] if rows == "T+1" else obs
    exp = d["obs"] if tdt == torch.float64 else d["obs"].astype(np.float32)
    np.testing.assert_array_equal(got.permute(1, 0, 2, 3).cpu().numpy(), exp)
    r = rew.cpu().numpy()
    r = r[..., None] if r.ndim == 2 else r
    np.testing.assert_array_equal(np.transpose(r, (1, 0, 2)), d["reward"][..., :r.shape[-1]])
    env.close()


@pytest.mark.parametrize("cfg,n,flags", [("C4", 131072, 0x6000), ("C3", 262144, 0x2000), ("C2", 1 << 20, 0x2000),
                                         ("C2", 262144, 0x6000)])
def test_default_store_policy_by_batch_size(cfg, n, flags):
    """IMENV_STORE_DEFAULT writes observations / rewards through at every size and the state rows too
    only while a launch's observation + reward bytes stay within 24 MiB (C4 at 131,072 envs: 13.6 MB;
    C2 at 262,144: 14.7 MB; not C3 at 262,144: 27.3 MB, nor C2 at 2^20: 58.7 MB)."""
    import bench
    from imenv import VectorInvEnv
    kind, c = bench.CONFIGS[cfg][:2]
    env = VectorInvEnv(kind, c, n_envs=n, device=DEV)
    env.reset()
    env.step(torch.zeros((n, env.N), device=DEV))
    got = int(re.search(r"flags=0x([0-9a-f]+)", env.kernel_info()).group(1), 16)
    assert got & 0x6800 == flags, env.kernel_info()
    env.close()


@pytest.mark.parametrize("config,n", [("C4", 131072), ("C2", 131072), ("C2", 262144)])
def test_gpu_launch_size_block_choice_is_invisible(config, n, monkeypatch):
    """Launches of at most two waves per SIMD (n <= 131,072) take 64-env blocks (JitFlags::small_blocks),
    larger ones 256; IMENV_JIT_BS forces either. One whole episode (in-kernel Philox demand, write-through
    stores) under each block size gives the same observations, rewards and state bit for bit."""
    import bench
    from imenv import VectorInvEnv
    kind, cfg = bench.CONFIGS[config][:2]
    runs = []
    for bs in (None, "64", "256"):
        if bs is None:
            monkeypatch.delenv("IMENV_JIT_BS", raising=False)
        else:
            monkeypatch.setenv("IMENV_JIT_BS", bs)
        monkeypatch.setenv("IMENV_JIT_STRICT", "1")
        env = VectorInvEnv(kind, cfg, n_envs=n, device=DEV)
        g = torch.Generator(device=DEV)
        g.manual_seed(7)
        T, N = env.T, env.N
        acts = torch.rand((T, n, N), generator=g, device=DEV) * 2 - 1
        obs = [env.reset().clone()]
        rews = []
        for t in range(T):
            o, r, _, _ = env.step(acts[t])
            obs.append(o.clone())
            rews.append(r.clone())
        info = env.kernel_info()
        s = env.state()
        st = [s["inv"].clone(), s["backlog"].clone(), s["order_u"].clone()]
        runs.append((int(re.search(r"bs=(\d+)", info).group(1)), torch.stack(obs), torch.stack(rews), st))
        env.close()
    assert runs[0][0] == (64 if n <= 131072 else 256), runs[0][0]
    assert (runs[1][0], runs[2][0]) == (64, 256)
    for bs, o, r, st in runs[1:]:
        assert torch.equal(o, runs[0][1]) and torch.equal(r, runs[0][2]), bs
        for a, b in zip(st, runs[0][3]):
            assert torch.equal(a, b), bs

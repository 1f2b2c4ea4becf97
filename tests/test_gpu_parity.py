"""HIP kernel parity: GPU step()/reset() vs the reference's golden vectors and the oracle.

All comparisons are exact: integer state/intermediates bit-equal; float64 obs and
rewards bit-equal to the reference's float64 (IEEE ops in the reference's order,
no FMA contraction); float32 obs equal to float32(reference obs).

Every test runs twice: with the hipRTC-specialised step kernel ("jit", the default path) and with
the ahead-of-time kernels ("aot"). IMENV_JIT_STRICT=1 makes a JIT failure an error, not a fallback.
"""
import os

import numpy as np
import pytest
import torch

from golden_io import case_names, fuzz_case_names, load_case
from oracle import philox
from oracle.im_oracle import OracleEnv

pytestmark = pytest.mark.gpu

CASES = case_names()
FUZZ = fuzz_case_names()     # randomly drawn configurations, reference outputs (tools/gen_fuzz_fixtures.py)
DEV = "cuda:0"
os.environ["IMENV_JIT_STRICT"] = "1"
MODE = {"kernel": "jit"}


@pytest.fixture(autouse=True, params=["jit", "aot"])
def kernel_mode(request):
    MODE["kernel"] = request.param
    yield request.param


def _env(kind, cfg, n, **kw):
    from imenv import VectorInvEnv
    env = VectorInvEnv(kind, cfg, n_envs=n, device=DEV, **kw)
    env.set_jit(1 if MODE["kernel"] == "jit" else 0)
    return env


def run_gpu_case(meta, d, obs_dtype=torch.float64, action_dtype=torch.float64):
    kind, cfg, E, T = meta["kind"], meta["config"], meta["E"], meta["T"]
    env = _env(kind, cfg, E, obs_dtype=obs_dtype)
    serial = kind in ("IM", "MAIM")
    dem = d["customer_demand"]
    noisy = meta["noisy"]
    obs0 = env.reset(customer_demand=dem[:, 0, :] if serial else dem, noisy_delay=bool(noisy),
                     noisy_delay_threshold=noisy, delay_uniforms=d["delay_uniforms"] if noisy else None)
    out = {k: [] for k in ("order", "demand", "acquisition", "ship", "inv", "backlog", "order_u", "obs",
                           "reward", "profit", "ship_to", "backlog_to")}
    obs0 = obs0.cpu().numpy()
    for t in range(T):
        a = torch.as_tensor(d["actions"][:, t, :], dtype=action_dtype, device=DEV)
        obs, rew, done, info = env.step(a, info=True)
        st = env.state()
        assert st["period"] == t + 1
        assert done == (t == T - 1)
        for k in ("order", "demand", "acquisition", "ship", "profit", "ship_to", "backlog_to"):
            out[k].append(info[k].cpu().numpy())
        for k in ("inv", "backlog", "order_u"):
            out[k].append(st[k].cpu().numpy())
        out["obs"].append(obs.cpu().numpy())
        r = rew.cpu().numpy()
        out["reward"].append(r if r.ndim == 2 else r[:, None])
    assert env.kernel_info().startswith(MODE["kernel"] + ":"), env.kernel_info()
    flags, anyv = env.errors()
    env.close()
    return obs0, {k: np.stack(v, axis=1) for k, v in out.items()}, anyv


@pytest.mark.parametrize("name", CASES + FUZZ)
def test_gpu_matches_reference_golden(name):
    meta, d = load_case(name)
    obs0, out, anyerr = run_gpu_case(meta, d)
    assert anyerr == 0
    np.testing.assert_array_equal(obs0, d["obs0"], err_msg="%s/obs0" % name)
    keys = ["order", "demand", "acquisition", "ship", "inv", "backlog", "order_u", "profit", "obs"]
    if meta["kind"] in ("IM_div", "MAIM_div"):
        keys += ["ship_to", "backlog_to"]
    for k in keys:
        np.testing.assert_array_equal(out[k].astype(np.float64), d[k], err_msg="%s/%s" % (name, k))
    ref_r = d["reward"]
    if out["reward"].shape[-1] == 1:
        ref_r = ref_r[..., :1]
    np.testing.assert_array_equal(out["reward"], ref_r, err_msg="%s/reward" % name)


@pytest.mark.parametrize("name", ["C1_IM4", "C2_MAIM4", "C3_IM8", "C4_MAIM_div1", "MAIM_div2_share",
                                  "IM4_td_pd_pa_L2", "fuzz/fz01_MAIM", "fuzz/fz04_IM", "fuzz/fz19_MAIM_div"])
def test_gpu_float32_obs_is_rounded_reference(name):
    meta, d = load_case(name)
    obs0, out, _ = run_gpu_case(meta, d, obs_dtype=torch.float32)
    np.testing.assert_array_equal(out["obs"], d["obs"].astype(np.float32))
    np.testing.assert_array_equal(obs0, d["obs0"].astype(np.float32))


C2 = dict(num_stages=4, num_periods=30, init_inv=np.ones(4) * 10, inv_target=np.zeros(4),
          inv_max=np.ones(4) * 30, price=np.array([5, 4, 3, 2, 1]),
          stock_cost=np.array([0.35, 0.3, 0.4, 0.2]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.9]),
          delay=np.array([1, 2, 3, 1]), demand_dist="poisson", mu=5, seed=52, independent=False)
C3 = dict(num_stages=8, num_periods=30, init_inv=np.ones(8) * 10, inv_target=np.zeros(8),
          inv_max=np.ones(8) * 30, price=np.array([9, 8, 7, 6, 5, 4, 3, 2, 1]),
          stock_cost=np.array([0.35, 0.3, 0.4, 0.2, 0.35, 0.3, 0.4, 0.2]),
          backlog_cost=np.array([0.5, 0.7, 0.6, 0.9, 0.5, 0.7, 0.6, 0.9]),
          delay=np.array([1, 2, 3, 1, 4, 2, 3, 1]), demand_dist="poisson", mu=5, seed=52)
C4 = dict(num_nodes=4, connections={0: [1], 1: [2, 3], 2: [], 3: []}, num_periods=30,
          init_inv=np.ones(4) * 10, inv_target=np.zeros(4), inv_max=np.ones(4) * 30,
          stock_cost=np.array([0.35, 0.3, 0.4, 0.4]), backlog_cost=np.array([0.5, 0.7, 0.6, 0.6]),
          delay=np.array([1, 2, 1, 1]), demand_dist="poisson", mu=5, seed=52, time_dependency=True,
          prev_demand=True, independent=False)


@pytest.mark.parametrize("kind,cfg,n", [("MAIM", C2, 8192), ("IM", C3, 4096), ("MAIM_div", C4, 8192),
                                         ("MAIM_div", dict(C4, noisy_demand=True, noisy_demand_threshold=0.3,
                                                           demand_dist="uniform", lower_upper=(1, 9)), 4096),
                                         ("IM", dict(C3, demand_dist="uniform", lower_upper=(2, 13)), 4096),
                                         ("MAIM", dict(C2, mu=12.5, independent=True), 4096),
                                         ("IM_div", dict(C4, mu=37.0, time_dependency=False), 4096),
                                         # wider drawn-demand tables: int16 (noisy uniform up to 2 x 399),
                                         # int32 (noisy uniform up to 2 x 19999)
                                         ("MAIM_div", dict(C4, noisy_demand=True, noisy_demand_threshold=0.3,
                                                           demand_dist="uniform", lower_upper=(100, 400)), 2048),
                                         ("IM_div", dict(C4, noisy_demand=True, noisy_demand_threshold=0.2,
                                                         demand_dist="uniform", lower_upper=(1, 20000),
                                                         time_dependency=False), 2048)])
@pytest.mark.parametrize("dtab", ["1", "0"])
def test_gpu_philox_rollout_matches_oracle(kind, cfg, n, dtab, monkeypatch):
    """Philox demand + f32 actions over two episodes == oracle with the same counters: drawn by the reset
    into the episode's table (dtab "1", imenv_draw_layout > 0) and drawn in the step kernel (dtab "0")."""
    monkeypatch.setenv("IMENV_DTAB", dtab)
    env = _env(kind, cfg, n, env_offset=1000)
    es = env.draw_layout()
    if dtab == "0":
        assert es == 0
    else:
        hi = cfg.get("lower_upper", (0, 0))[1] * (2 if cfg.get("noisy_demand") else 1)
        assert es == (4 if hi > 32767 else 2 if hi > 255 else 1)
    ora = OracleEnv(kind, cfg, n_envs=n)
    if cfg["demand_dist"] == "poisson":
        np.testing.assert_array_equal(env.poisson_table(), philox.poisson_thresholds(cfg.get("mu", 5)))
    rs = np.random.RandomState(7)
    for ep in range(2):
        env.reset()
        ora.reset(rng=dict(seed=52, episode=ep, env_offset=1000, dist=cfg["demand_dist"], mu=cfg.get("mu", 5),
                           lower_upper=cfg.get("lower_upper", (1, 5))))
        for t in range(30):
            a32 = rs.uniform(-1.1, 1.1, size=(n, env.N)).astype(np.float32)
            o_g, r_g, _, info = env.step(torch.as_tensor(a32, device=DEV), info=True)
            o_c, r_c, _, info_c = ora.step(a32.astype(np.float64))
            np.testing.assert_array_equal(info["demand"].cpu().numpy(), info_c["demand"], err_msg="t=%d" % t)
            st = env.state()
            for k in ("inv", "backlog", "order_u"):
                np.testing.assert_array_equal(st[k].cpu().numpy(), ora.state_arrays()[k])
            np.testing.assert_array_equal(o_g.cpu().numpy(), o_c.astype(np.float32))
            r_c = r_c if r_c.ndim == 2 else r_c
            np.testing.assert_array_equal(r_g.cpu().numpy(), r_c)


def test_gpu_philox_noisy_delay_matches_oracle():
    cfg = dict(C2, time_dependency=True)
    n = 4096
    env = _env("MAIM", cfg, n)
    ora = OracleEnv("MAIM", cfg, n_envs=n)
    env.reset(noisy_delay=True, noisy_delay_threshold=0.3)
    ora.reset(rng=dict(seed=52, episode=0, env_offset=0, mu=5), noisy_delay=True, noisy_delay_threshold=0.3)
    rs = np.random.RandomState(3)
    for t in range(30):
        a = rs.uniform(-1, 1, size=(n, 4))
        o_g, r_g, _, info = env.step(torch.as_tensor(a, device=DEV), info=True)
        o_c, r_c, _, info_c = ora.step(a)
        np.testing.assert_array_equal(info["acquisition"].cpu().numpy(), info_c["acquisition"])
        np.testing.assert_array_equal(o_g.cpu().numpy(), o_c.astype(np.float32))
        np.testing.assert_array_equal(r_g.cpu().numpy(), r_c)


def test_gpu_sharding_invariance():
    """Two handles at env_offset 0 and n/2 reproduce one handle of n envs (RNG keyed by global id)."""
    n = 1 << 14
    full = _env("MAIM", C2, n)
    halves = [_env("MAIM", C2, n // 2, env_offset=r * (n // 2)) for r in range(2)]
    full.reset()
    for h in halves:
        h.reset()
    g = torch.Generator(device="cpu").manual_seed(0)
    for t in range(30):
        a = (torch.rand((n, 4), generator=g) * 2 - 1).to(DEV)
        of, rf, _, _ = full.step(a)
        parts = [h.step(a[r * (n // 2):(r + 1) * (n // 2)]) for r, h in enumerate(halves)]
        assert torch.equal(of, torch.cat([p[0] for p in parts]))
        assert torch.equal(rf, torch.cat([p[1] for p in parts]))


def test_gpu_full_size_properties():
    """2^20 envs (the bench workload): invariants that hold at any size, plus demand statistics."""
    n = 1 << 20
    env = _env("MAIM", C2, n)
    env.reset()
    g = torch.Generator(device="cpu").manual_seed(1)
    im = torch.tensor(C2["inv_max"], device=DEV, dtype=torch.int32)
    dsum = torch.zeros((), dtype=torch.float64, device=DEV)
    dsq = torch.zeros((), dtype=torch.float64, device=DEV)
    counts = torch.zeros(64, dtype=torch.float64, device=DEV)
    for t in range(30):
        a = (torch.rand((n, 4), generator=g) * 2 - 1).to(DEV)
        inv0 = env.state()
        obs, rew, done, info = env.step(a, info=True)
        st = env.state()
        assert bool(((st["inv"] >= 0) & (st["inv"] <= im)).all())
        assert bool(((st["backlog"] >= 0) & (st["backlog"] <= im)).all())
        assert bool(((info["order"] >= 0) & (info["order"] <= im)).all())
        # balance: ship <= backlog + demand and ship <= inv + acquisition (IM_env.py:315)
        assert bool((info["ship"] <= inv0["backlog"] + info["demand"]).all())
        assert bool((info["ship"] <= inv0["inv"] + info["acquisition"]).all())
        # shared reward is the mean of per-stage profits
        prof = info["profit"]
        s = ((((torch.zeros(n, dtype=torch.float64, device=DEV) + prof[:, 0]) + prof[:, 1]) + prof[:, 2]) + prof[:, 3])
        assert torch.equal(rew, s / 4)
        assert bool((obs.abs() <= 1.0).all())
        dcur = info["demand"][:, 0].to(torch.float64)
        dsum += dcur.sum()
        dsq += (dcur * dcur).sum()
        counts += torch.bincount(info["demand"][:, 0].clamp(max=63).long(), minlength=64).double()
    m = (dsum / (30 * n)).item()
    v = (dsq / (30 * n)).item() - m * m
    # demand = min(Poisson(5), inv_max=30): mean/var of Poisson(5) to within sampling error
    assert abs(m - 5.0) < 0.01 and abs(v - 5.0) < 0.03
    from scipy.stats import poisson
    N = 30 * n
    exp = poisson.pmf(np.arange(64), 5) * N
    obs_c = counts.cpu().numpy()
    k = exp > 50
    chi2 = (((obs_c[k] - exp[k]) ** 2) / exp[k]).sum()
    assert chi2 < 3 * k.sum(), chi2


def test_gpu_errors_and_done():
    from imenv import ImEnvNativeError
    env = _env("MAIM", C2, 64)
    with pytest.raises(ImEnvNativeError):
        env.step(torch.zeros((64, 4), device=DEV))        # before reset
    env.reset()
    for _ in range(30):
        env.step(torch.zeros((64, 4), device=DEV))
    with pytest.raises(ImEnvNativeError):
        env.step(torch.zeros((64, 4), device=DEV))        # past the horizon (reference: IndexError)


@pytest.mark.parametrize("name", ["C2_MAIM4", "C4_MAIM_div1", "IM4_td_pd_pa_L2", "MAIM_div2_share",
                                  "IM4_noisy_delay"])
@pytest.mark.parametrize("state_bytes", ["2", "4"])
def test_gpu_wider_state_layouts_match_reference(name, state_bytes, monkeypatch):
    """The packed state uses the narrowest element type the spec's bounds allow (uint8 for these
    cases); forcing int16 / int32 rows must give the same bit-exact results."""
    monkeypatch.setenv("IMENV_STATE_BYTES", state_bytes)
    meta, d = load_case(name)
    from imenv import VectorInvEnv
    probe = VectorInvEnv(meta["kind"], meta["config"], n_envs=4, device=DEV)
    assert probe.state_layout()[0] == int(state_bytes)
    probe.close()
    obs0, out, anyerr = run_gpu_case(meta, d)
    assert anyerr == 0
    for k in ("order", "demand", "acquisition", "ship", "inv", "backlog", "order_u", "profit", "obs"):
        np.testing.assert_array_equal(out[k].astype(np.float64), d[k], err_msg="%s/%s" % (name, k))


def test_gpu_narrowest_layout_selected():
    from imenv import VectorInvEnv
    meta, _ = load_case("C2_MAIM4")
    env = VectorInvEnv(meta["kind"], meta["config"], n_envs=4, device=DEV)
    assert env.state_layout()[0] == 1          # every C2 value is provably <= 255
    env.close()
    meta, _ = load_case("MAIM3_defaults")      # inv_max 200: shipments can exceed 255
    env = VectorInvEnv(meta["kind"], meta["config"], n_envs=4, device=DEV)
    assert env.state_layout()[0] == 2
    env.close()


@pytest.mark.parametrize("name", ["C2_MAIM4", "C3_IM8", "IM_div1"])
def test_gpu_two_envs_per_thread_variant(name, kernel_mode, monkeypatch):
    """The JIT kernel's two-envs-per-thread layout (IMENV_JIT_EPT=2, staged float32 observations)
    computes the same function; 32 golden envs do not fill one 512-env block (ragged slabs)."""
    if kernel_mode != "jit":
        pytest.skip("JIT-only variant")
    monkeypatch.setenv("IMENV_JIT_EPT", "2")
    meta, d = load_case(name)
    obs0, out, _ = run_gpu_case(meta, d, obs_dtype=torch.float32)
    np.testing.assert_array_equal(out["obs"], d["obs"].astype(np.float32))
    for k in ("inv", "backlog", "order_u"):
        np.testing.assert_array_equal(out[k].astype(np.float64), d[k])


C2_3 = dict(C2, num_stages=3, init_inv=np.ones(3) * 10, inv_target=np.zeros(3), inv_max=np.ones(3) * 30,
            price=np.array([4, 3, 2, 1]), stock_cost=np.array([0.35, 0.3, 0.4]),
            backlog_cost=np.array([0.5, 0.7, 0.6]), delay=np.array([1, 2, 3]))


@pytest.mark.parametrize("kind,cfg", [("MAIM", C2), ("IM", C3), ("MAIM_div", C4), ("MAIM", C2_3),
                                      ("IM", dict(C2, time_dependency=True, prev_demand=True, prev_actions=True,
                                                  prev_length=2))])
@pytest.mark.parametrize("odt", [torch.float32, torch.float64])
def test_gpu_ragged_env_counts(kind, cfg, odt):
    """Env counts that fill no block exactly (1, 3, 255, 257, 1000: tail lanes, partial LDS obs slabs
    whose value count is not a multiple of the float4 / double2 run; 3 stages: odd base rows) == oracle,
    float32 actions, float32 / float64 observations, in-kernel draws."""
    cast = (lambda x: x.astype(np.float32)) if odt == torch.float32 else (lambda x: x)
    for n in (1, 3, 255, 257, 1000):
        env = _env(kind, cfg, n, env_offset=77, obs_dtype=odt)
        ora = OracleEnv(kind, cfg, n_envs=n)
        o_g = env.reset()
        o_c = ora.reset(rng=dict(seed=52, episode=0, env_offset=77, mu=5))
        np.testing.assert_array_equal(o_g.cpu().numpy(), cast(o_c))
        rs = np.random.RandomState(n)
        for t in range(30):
            a32 = rs.uniform(-1, 1, size=(n, env.N)).astype(np.float32)
            o_g, r_g, d_g, _ = env.step(torch.as_tensor(a32, device=DEV))
            o_c, r_c, d_c, _ = ora.step(a32.astype(np.float64))
            np.testing.assert_array_equal(o_g.cpu().numpy(), cast(o_c), err_msg="n=%d t=%d" % (n, t))
            np.testing.assert_array_equal(r_g.cpu().numpy(), r_c, err_msg="n=%d t=%d" % (n, t))
            st = env.state()
            for k in ("inv", "backlog", "order_u"):
                np.testing.assert_array_equal(st[k].cpu().numpy(), ora.state_arrays()[k])
        env.close()


IM10 = dict(num_stages=10, num_periods=30, init_inv=np.ones(10) * 10, inv_target=np.zeros(10),
            inv_max=np.ones(10) * 30, price=np.arange(11, 0, -1), stock_cost=np.full(10, 0.3),
            backlog_cost=np.full(10, 0.6), delay=np.array([1, 2, 3, 1, 4, 2, 3, 1, 2, 2]), demand_dist="poisson",
            mu=5, seed=52)


@pytest.mark.parametrize("state_bytes", [None, "2", "4"])
def test_gpu_jit_and_aot_continue_each_others_episode(state_bytes, monkeypatch):
    """10 stages (the AOT kernel pads them to 16: element-wise rows) with noisy delay (int16 / int32
    carry rows): the JIT and AOT kernels alternate step by step within one episode, so every packed
    row (net inventory, order_u, carry) must have one layout for both. == oracle, in-kernel draws."""
    if state_bytes:
        monkeypatch.setenv("IMENV_STATE_BYTES", state_bytes)
    n = 300
    env = _env("IM", IM10, n, env_offset=5)
    ora = OracleEnv("IM", IM10, n_envs=n)
    for ep in range(2):
        o_g = env.reset(noisy_delay=True, noisy_delay_threshold=0.4)
        o_c = ora.reset(noisy_delay=True, noisy_delay_threshold=0.4,
                        rng=dict(seed=52, episode=ep, env_offset=5, mu=5))
        np.testing.assert_array_equal(o_g.cpu().numpy(), o_c.astype(np.float32))
        rs = np.random.RandomState(ep)
        for t in range(30):
            env.set_jit((t + ep) % 2)
            a = rs.uniform(-1, 1, size=(n, 10))
            o_g, r_g, _, _ = env.step(torch.as_tensor(a, device=DEV))
            o_c, r_c, _, _ = ora.step(a)
            np.testing.assert_array_equal(o_g.cpu().numpy(), o_c.astype(np.float32), err_msg="ep %d t %d" % (ep, t))
            np.testing.assert_array_equal(r_g.cpu().numpy(), r_c, err_msg="ep %d t %d" % (ep, t))
            st = env.state()
            for k in ("inv", "backlog", "order_u"):
                np.testing.assert_array_equal(st[k].cpu().numpy(), ora.state_arrays()[k])
        assert ("jit:" in env.kernel_info()) == ((29 + ep) % 2 == 1)
    env.close()


def test_gpu_step_traffic_matches_bench_formula():
    """Algorithmic bytes per env-step for the bench layouts: C2 96 B steady,
    95.5 B averaged over the 30-period episode (t = 0 reads no state rows, node i no arrival
    before t = d_i). The drawn-demand table (imenv_draw_layout: small handles) is counted only with
    handover=True: + one byte per retailer read at t % 4 != 0 and three written at t % 4 == 0 (periods
    t+1..t+3: 22 + 22 bytes over the episode)."""
    env = _env("MAIM", C2, 64)
    assert env.state_layout()[0] == 1
    dt = env.draw_layout()
    assert dt == (0 if os.environ.get("IMENV_DTAB") == "0" else 1)
    steady, avg = env.step_traffic()
    assert steady == 96 and abs(avg - (96 - 15 / 30)) < 1e-9
    steady, avg = env.step_traffic(handover=True)
    assert steady == 96 + dt and abs(avg - (96 + dt * 44 / 30 - 15 / 30)) < 1e-9
    env.close()
    env = _env("MAIM_div", C4, 64)     # td slot of node 1 (delay 2), backlog_to rows, no history rows
    steady, _ = env.step_traffic()
    # backlog_to of the two split children only (imenv_split_layout): int16 (T x order_max = 900 fits),
    # 4 B read + 4 B written; int32 under IMENV_BTO_BYTES=4
    nb, be = env.split_layout()
    assert nb == 2 and be == (4 if os.environ.get("IMENV_BTO_BYTES") == "4" else 2)
    # two retailers: no drawn-demand table by default (imenv_draw_layout; capi dtab_es_for)
    assert env.draw_layout() == (1 if os.environ.get("IMENV_DTAB") == "1" else 0)
    assert steady == 16 + 16 + 4 + 1 + 4 + 2 * nb * be + 96 + 8
    assert env.step_traffic(handover=True)[0] == steady + env.draw_layout() * env.spec.num_retailers
    env.close()


def test_gpu_output_buffers_are_checked_before_launch():
    """Caller-owned obs / reward buffers of the wrong shape, dtype or device raise before any kernel
    writes into them (a short buffer would otherwise be written out of bounds)."""
    env = _env("MAIM", C2, 256)
    obs0 = torch.empty((256, 4, 3), dtype=torch.float32, device=DEV)
    env.reset(obs_out=obs0)
    a = torch.zeros((256, 4), device=DEV)
    for bad in (torch.empty((255, 4, 3), device=DEV), torch.empty((256, 4, 3), dtype=torch.float16, device=DEV),
                torch.empty((256, 4, 3)), torch.empty((256, 3, 4), device=DEV).transpose(1, 2)):
        with pytest.raises(ValueError):
            env.step(a, obs_out=bad)
    with pytest.raises(ValueError):
        env.step(a, reward_out=torch.empty(256, dtype=torch.float32, device=DEV))
    with pytest.raises(ValueError):
        env.reset(obs_out=torch.empty((128, 4, 3), device=DEV))
    assert env.state()["period"] == 0        # nothing was launched by the rejected calls
    env.close()


@pytest.mark.parametrize("kind,cfg", [("MAIM", dict(C2, demand_dist="custom")), ("IM", dict(C3, demand_dist="custom")),
                                      ("MAIM_div", dict(C4, demand_dist="custom")),
                                      ("IM", dict(C3, demand_dist="custom", customer_demand=np.arange(30) % 7)),
                                      ("MAIM_div", dict(C4, demand_dist="custom",
                                                        customer_demand=np.arange(60).reshape(2, 30) % 9))])
def test_gpu_custom_demand_from_config(kind, cfg):
    """demand_dist "custom" with reset() and no demand argument: the config's customer_demand, or the
    reference's default of 5 per period ([T] serial, IM_env.py:189; [R, T] tree, IM_div_env.py:226),
    for every env of a batch."""
    n = 64
    env = _env(kind, cfg, n)
    ora = OracleEnv(kind, cfg, n_envs=n)
    serial = kind in ("IM", "MAIM")
    T = env.T
    dem = cfg.get("customer_demand", np.ones(T) * 5 if serial else np.ones((2, T)) * 5)
    dem = np.broadcast_to(np.asarray(dem)[None], (n,) + np.asarray(dem).shape)
    o0 = env.reset()
    r0 = ora.reset(customer_demand=dem)
    np.testing.assert_array_equal(o0.cpu().numpy().astype(np.float64), r0.astype(np.float32))
    rs = np.random.RandomState(3)
    for t in range(T):
        a = rs.uniform(-1, 1, size=(n, env.N))
        obs, rew, _, info = env.step(torch.as_tensor(a, device=DEV), info=True)
        ro, rr, _, rinfo = ora.step(a)
        np.testing.assert_array_equal(info["demand"].cpu().numpy().astype(np.float64), rinfo["demand"])
        np.testing.assert_array_equal(obs.cpu().numpy(), ro.astype(np.float32))
        np.testing.assert_array_equal(rew.cpu().numpy(), rr)
    env.close()


def test_gpu_huge_batch_matches_oracle_on_slices():
    """2^26 envs in one handle (64x the bench size; 3.2 GB of observations per step): env ranges at
    the start, middle and end of the batch equal the oracle with the same Philox keys over a whole
    episode (in-kernel demand, float32 actions)."""
    n = 1 << 26
    env = _env("MAIM", C2, n)
    slices = [(0, 256), (n // 2 - 100, 256), (n - 256, 256)]
    oras = [OracleEnv("MAIM", C2, n_envs=k) for _, k in slices]
    o0 = env.reset()
    for (s, k), ora in zip(slices, oras):
        r0 = ora.reset(rng=dict(seed=52, episode=0, env_offset=s, dist="poisson", mu=5))
        np.testing.assert_array_equal(o0[s:s + k].cpu().numpy(), r0.astype(np.float32))
    g = torch.Generator(device=DEV)
    g.manual_seed(11)
    for t in range(30):
        a = torch.rand((n, 4), generator=g, device=DEV) * 2.2 - 1.1
        obs, rew, _, _ = env.step(a)
        for (s, k), ora in zip(slices, oras):
            o_c, r_c, _, _ = ora.step(a[s:s + k].double().cpu().numpy())
            np.testing.assert_array_equal(obs[s:s + k].cpu().numpy(), o_c.astype(np.float32), err_msg="t=%d" % t)
            np.testing.assert_array_equal(rew[s:s + k].cpu().numpy(), r_c)
    env.close()

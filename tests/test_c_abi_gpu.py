"""The C ABI driven from C++ alone (examples/c_abi_episode.cpp, built by __graft_entry__.build()):
hipMalloc'd buffers, imenv_create / imenv_reset / imenv_step / imenv_kernel_info, no Python or
torch in the process. On the reference's golden cases (per-env host demand, float64 actions and
observations, host-fed noisy-delay uniforms where the case has them) its outputs equal the
reference's bit for bit; stepping past the horizon returns an
error code (the reference raises IndexError)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from golden_io import load_case

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "examples", "bin", "c_abi_episode")


@pytest.mark.parametrize("name", ["C2_MAIM4", "C3_IM8", "C4_MAIM_div1", "MAIM4_indep", "IM4_td_pd_pa_L2",
                                  "MAIM_div1_noisy_delay", "fuzz/fz04_IM", "fuzz/fz19_MAIM_div",
                                  "fuzz/fz25_MAIM_div_pd_only"])
def test_cpp_host_reproduces_reference_golden(name, tmp_path):
    from imenv import _native as nat
    from imenv import build_spec
    if not os.path.exists(BIN):
        pytest.fail("examples/bin/c_abi_episode not built (python __graft_entry__.py build)")
    meta, d = load_case(name)
    hs = build_spec(meta["kind"], meta["config"])
    spec = hs.to_c()
    E, T = meta["E"], meta["T"]
    N, F = d["obs"].shape[2], d["obs"].shape[3]
    dem = d["customer_demand"]                      # [E, R, T]
    R = dem.shape[1]
    rc = N if hs.reward_mode == nat.REWARD_INDEPENDENT else 1
    (tmp_path / "spec.bin").write_bytes(ctypes.string_at(ctypes.addressof(spec), ctypes.sizeof(spec)))
    noisy = float(meta["noisy"])
    (tmp_path / "dims.txt").write_text("%d %d %d %d %d %d %r\n" % (E, T, N, F, R, rc, noisy))
    if noisy:     # host-fed noisy-delay uniforms, [E, T, N] -> [T][N][n]
        np.ascontiguousarray(d["delay_uniforms"].transpose(1, 2, 0), dtype=np.float64).tofile(tmp_path / "delay_u.f64")
    np.ascontiguousarray(dem.transpose(2, 1, 0), dtype=np.int32).tofile(tmp_path / "demand.i32")
    np.ascontiguousarray(d["actions"].transpose(1, 0, 2), dtype=np.float64).tofile(tmp_path / "actions.f64")
    r = subprocess.run([BIN, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    obs0 = np.fromfile(tmp_path / "obs0.f64").reshape(E, N, F)
    obs = np.fromfile(tmp_path / "obs.f64").reshape(T, E, N, F)
    rew = np.fromfile(tmp_path / "reward.f64").reshape(T, E, rc)
    np.testing.assert_array_equal(obs0, d["obs0"])
    np.testing.assert_array_equal(obs.transpose(1, 0, 2, 3), d["obs"])
    np.testing.assert_array_equal(rew.transpose(1, 0, 2), d["reward"][..., :rc])
    lines = (tmp_path / "done.txt").read_text().splitlines()
    assert lines[0].split() == ["0"] * (T - 1) + ["1"]
    assert lines[1] == "past_horizon_rc %d" % nat.E_DONE
    # default store policy: write-through; float64 observations have a kernel name of their own
    assert lines[2].startswith("jit:imenv_step_jit_wt_o64["), lines[2]


PLAN_BIN = os.path.join(ROOT, "examples", "bin", "c_abi_plan")


@pytest.mark.parametrize("name", ["SHLP8", "SHLP_div1", "SHLP_div2"])
def test_cpp_host_plan_replay_reproduces_reference_golden(name, tmp_path):
    """examples/c_abi_plan.cpp: one imenv_plan_rollout call from C++ replays every scenario's own plan
    and returns the LP scripts' per-step rewards and sums, equal to the reference loop's bit for bit."""
    from golden_io import load_base_stock
    from imenv import build_spec
    if not os.path.exists(PLAN_BIN):
        pytest.fail("examples/bin/c_abi_plan not built (python __graft_entry__.py build)")
    meta, cases = load_base_stock("plan_replay.npz")
    m, d = meta[name], cases[name]
    assert m["layout"] == "episode" and d["plans"].shape[1] == 1
    spec = build_spec(m["kind"], m["config"]).to_c()
    T, _, S, N = d["plans"].shape
    dem = d["demand"] if d["demand"].ndim == 3 else d["demand"][:, None, :]     # [S, R, T]
    R = dem.shape[1]
    (tmp_path / "spec.bin").write_bytes(ctypes.string_at(ctypes.addressof(spec), ctypes.sizeof(spec)))
    (tmp_path / "dims.txt").write_text("%d %d %d %d\n" % (S, T, N, R))
    np.ascontiguousarray(dem.transpose(2, 1, 0), dtype=np.int32).tofile(tmp_path / "demand.i32")
    np.ascontiguousarray(d["plans"][:, 0], dtype=np.float64).tofile(tmp_path / "plans.f64")
    r = subprocess.run([PLAN_BIN, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rew = np.fromfile(tmp_path / "rewards.f64").reshape(T, S)
    st = np.fromfile(tmp_path / "stats.f64").reshape(5, S)
    np.testing.assert_array_equal(rew, d["rewards"][:, 0])
    for j, k in ((0, "return"), (2, "inventory"), (3, "backlog"), (4, "customer_backlog")):
        np.testing.assert_array_equal(st[j], d[k][0], err_msg=k)
    ms = np.fromfile(tmp_path / "mean_std.f64").reshape(5, 2)
    np.testing.assert_allclose(ms[0], [np.mean(d["return"][0]), np.std(d["return"][0])], rtol=1e-12)
    assert "rollout jit:imenv_rollout_jit[" in (tmp_path / "info.txt").read_text()

"""Centralised-critic observation builder: oracle vs the reference's central_critic_observer
(tests/golden/cc_obs.npz, tools/gen_cc_fixtures.py), then the HIP kernel (imenv_cc_observation)
vs both, bit for bit, for f32 / f64 observations and actions."""
import os

import numpy as np
import pytest

from golden_io import GOLDEN
from oracle.cc_obs import cc_observation as cc_ref

Z = np.load(os.path.join(GOLDEN, "cc_obs.npz"), allow_pickle=False)
NAMES = sorted({k.split("/")[0] for k in Z.files})


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference_observer(name):
    obs, act, cc = Z[name + "/obs"], Z[name + "/actions"], Z[name + "/cc"]
    E, T, N, F = obs.shape
    got = cc_ref(obs.reshape(E * T, N, F), act.reshape(E * T, N)).reshape(cc.shape)
    np.testing.assert_array_equal(got, cc)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("odt,adt", [("f64", "f64"), ("f32", "f32"), ("f32", "f64"), ("f64", "f32")])
def test_gpu_cc_observation(name, odt, adt):
    import torch
    from imenv.critic import cc_observation, split_cc_observation
    dt = {"f32": torch.float32, "f64": torch.float64}
    obs, act, cc = Z[name + "/obs"], Z[name + "/actions"], Z[name + "/cc"]
    o = torch.as_tensor(obs, dtype=dt[odt], device="cuda:0")
    a = torch.as_tensor(act, dtype=dt[adt], device="cuda:0")
    got = cc_observation(o, a).cpu().numpy()
    exp = cc_ref(o.cpu().numpy().reshape(-1, *obs.shape[2:]), a.cpu().numpy().reshape(-1, obs.shape[2]))
    exp = exp.reshape(got.shape)
    np.testing.assert_array_equal(got, exp)
    if odt == "f64" and adt == "f64":
        np.testing.assert_array_equal(got, cc)
    parts = split_cc_observation(torch.as_tensor(got), obs.shape[-1])
    np.testing.assert_array_equal(parts["own_obs"].numpy(), o.cpu().numpy())
    z = cc_observation(o).cpu().numpy()          # no actions: zeros, as the observer leaves them
    assert not z[..., :obs.shape[2] - 1].any()


@pytest.mark.gpu
def test_gpu_cc_observation_rollout_buffer():
    """A [T, n] rollout buffer of 30 x 65,536 MAIM 4-stage observations in one call."""
    import torch
    from imenv.critic import cc_observation
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1)
    obs = torch.rand((30, 65536, 4, 3), generator=g, device="cuda:0") * 2 - 1
    act = torch.rand((30, 65536, 4), generator=g, device="cuda:0") * 3 - 1.5
    got = cc_observation(obs, act)
    assert got.shape == (30, 65536, 4, 15)
    sl = slice(0, 30000, 997)
    exp = cc_ref(obs[:, sl].reshape(-1, 4, 3).cpu().numpy(), act[:, sl].reshape(-1, 4).cpu().numpy())
    np.testing.assert_array_equal(got[:, sl].reshape(-1, 4, 15).cpu().numpy(), exp)


@pytest.mark.gpu
@pytest.mark.parametrize("N,F", [(2, 1), (3, 3), (4, 3), (5, 2), (8, 7), (16, 4), (16, 12)])
@pytest.mark.parametrize("dt", ["f32", "f64"])
@pytest.mark.parametrize("bs", ["256", "512"])
def test_gpu_cc_observation_shapes(N, F, dt, bs, monkeypatch):
    """Staged (env, agent)-row kernel (blocks of 256 // N envs: ragged when N does not divide 256, odd
    and even row lengths; IMENV_CC_BS=512 runs the 512-thread variant, read on every call) and, for
    rows too wide for its 48 KiB slab (16 agents x 12 features), the element-wise kernel; env counts
    that leave a partial last block. NaN and infinite actions clip as np.clip does (NaN passes
    through). Bit-exact vs the oracle."""
    import torch
    from imenv.critic import cc_observation
    monkeypatch.setenv("IMENV_CC_BS", bs)
    tdt = {"f32": torch.float32, "f64": torch.float64}[dt]
    g = torch.Generator(device="cuda:0")
    g.manual_seed(N * 100 + F)
    for n in (1, 7, 1000, 4099):
        obs = (torch.rand((n, N, F), generator=g, device="cuda:0", dtype=torch.float64) * 4 - 2).to(tdt)
        act = (torch.rand((n, N), generator=g, device="cuda:0", dtype=torch.float64) * 3 - 1.5).to(tdt)
        if n >= 7:
            act.view(-1)[[1, 5]] = float("nan")
            act.view(-1)[2] = float("inf")
            act.view(-1)[3] = -float("inf")
        got = cc_observation(obs, act).cpu().numpy()
        np.testing.assert_array_equal(got, cc_ref(obs.cpu().numpy(), act.cpu().numpy()), err_msg="n=%d" % n)

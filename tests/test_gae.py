"""GAE (imenv_gae) vs the restated RLlib compute_advantages (oracle/gae.py, scipy lfilter).

Bit-exact float32 outputs for completed trajectories (float64 arithmetic, the reference's path when
last_r = 0.0) and with bootstrap values; float32 / float64 rewards and values; a full-size
[30, 2^20] buffer checked on sampled envs. The reference's own RLlib is absent: parity unpinned vs
RLlib itself, pinned to its published algorithm."""
import numpy as np
import pytest

from oracle.gae import compute_advantages, gae_batch


def test_oracle_discount_cumsum_recursion():
    """The lfilter recursion the kernel restates: adv_t = c * adv_{t+1} + delta_t in float64."""
    rs = np.random.RandomState(0)
    r = rs.standard_normal(30).astype(np.float32) * 40
    v = rs.standard_normal(30).astype(np.float32) * 90
    adv, vt = compute_advantages(r, v, 0.0, 0.99, 0.95)
    vp = np.concatenate([v.astype(np.float64), [0.0]])
    c = 0.99 * 0.95
    a = np.zeros(30)
    for t in range(29, -1, -1):
        d = (np.float64(r[t]) + 0.99 * vp[t + 1]) - vp[t]
        a[t] = 0.0 + d if t == 29 else c * a[t + 1] + d
    np.testing.assert_array_equal(adv, a.astype(np.float32))
    np.testing.assert_array_equal(vt, (a + v).astype(np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("rdt,vdt,boot", [("f32", "f32", False), ("f64", "f32", False), ("f64", "f64", True),
                                          ("f32", "f32", True)])
def test_gpu_gae_matches_oracle(rdt, vdt, boot):
    import torch
    from imenv.rollout import gae
    dt = {"f32": (torch.float32, np.float32), "f64": (torch.float64, np.float64)}
    rs = np.random.RandomState(1)
    T, n = 30, 3000
    r = (rs.standard_normal((T, n)) * 50).astype(dt[rdt][1])
    v = (rs.standard_normal((T, n)) * 200).astype(dt[vdt][1])
    lv = (rs.standard_normal(n) * 200).astype(dt[vdt][1]) if boot else None
    adv, vt = gae(torch.as_tensor(r, device="cuda:0"), torch.as_tensor(v, device="cuda:0"),
                  torch.as_tensor(lv, device="cuda:0") if boot else None)
    ea, ev = gae_batch(r, v, lv)
    np.testing.assert_array_equal(adv.cpu().numpy(), ea)
    np.testing.assert_array_equal(vt.cpu().numpy(), ev)


@pytest.mark.gpu
def test_gpu_gae_full_size_buffer():
    import torch
    from imenv.rollout import gae
    T, n = 30, 1 << 20
    g = torch.Generator(device="cuda:0")
    g.manual_seed(2)
    r = torch.randn((T, n), generator=g, device="cuda:0", dtype=torch.float64) * 30
    v = torch.randn((T, n), generator=g, device="cuda:0") * 100
    adv, vt = gae(r, v)
    idx = np.arange(0, n, 4099)
    ea, ev = gae_batch(r[:, idx].cpu().numpy(), v[:, idx].cpu().numpy())
    np.testing.assert_array_equal(adv[:, idx].cpu().numpy(), ea)
    np.testing.assert_array_equal(vt[:, idx].cpu().numpy(), ev)


@pytest.mark.gpu
def test_rollout_buffer_with_env():
    """VectorInvEnv writes obs / rewards into the buffer in place; advantages come out of one launch."""
    import torch
    import gen_cfg
    from imenv import VectorInvEnv
    from imenv.rollout import RolloutBuffer
    env = VectorInvEnv("MAIM", gen_cfg.serial4(independent=False), n_envs=4096, device="cuda:0")
    buf = RolloutBuffer(env)
    buf.obs[0] = env.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    for t in range(env.T):
        buf.actions[t] = torch.rand((env.n, env.N), generator=g, device="cuda:0") * 2 - 1
        buf.values[t] = buf.obs[t].mean(dim=(1, 2)) * 10
        env.step(buf.actions[t], obs_out=buf.obs[t + 1], reward_out=buf.rewards[t])
    adv, vt = buf.advantages()
    ea, ev = gae_batch(buf.rewards.cpu().numpy(), buf.values.cpu().numpy())
    np.testing.assert_array_equal(adv.cpu().numpy(), ea)
    np.testing.assert_array_equal(vt.cpu().numpy(), ev)
    # the buffer's own launcher (RolloutBuffer.step -> rollout_stepper) fills a second buffer identically
    env2 = VectorInvEnv("MAIM", gen_cfg.serial4(independent=False), n_envs=4096, device="cuda:0")
    buf2 = RolloutBuffer(env2)
    env2.reset(obs_out=buf2.obs[0])
    buf2.actions.copy_(buf.actions)
    for t in range(env2.T):
        assert buf2.step(t) == (t == env2.T - 1)
    assert torch.equal(buf2.obs, buf.obs) and torch.equal(buf2.rewards, buf.rewards)
    with pytest.raises(AttributeError):       # the stepper holds these tensors: no rebinding
        buf2.actions = torch.zeros_like(buf2.actions)
    env.close()
    env2.close()

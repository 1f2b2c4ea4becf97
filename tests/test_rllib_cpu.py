"""The batched RLlib surfaces' host logic on CPU (imenv/rllib.py): RLlib's call sequences (VectorEnv:
vector_reset / vector_step / reset_at; BaseEnv: poll / send_actions / try_reset), the dict shapes and
release order RLlib's own _MultiAgentEnvToBaseEnv uses, lockstep resets and their refusals. The
device is replaced by a test-only stand-in that runs the oracle behind VectorInvEnv's methods, so the
golden reference sessions (tests/golden) pin the values here as they do on the GPU
(tests/test_rllib_gpu.py runs the same sequences on the real kernel)."""
import numpy as np
import pytest
import torch

from golden_io import load_case
from oracle.im_oracle import OracleEnv


class OracleVectorEnv:
    """Test-only stand-in for VectorInvEnv: the oracle (oracle/im_oracle.py) behind the same calls."""

    def __init__(self, spec, n_envs=1, device=None, env_offset=0, obs_dtype=torch.float32):
        self.spec = spec
        self.ora = OracleEnv(spec.kind, spec.config, n_envs=n_envs)
        self.n, self.N, self.F, self.T = n_envs, self.ora.N, spec.num_features, spec.num_periods
        self.device = torch.device("cpu")
        self.period, self.episode = 0, -1

    def reset(self, customer_demand=None, noisy_delay=False, noisy_delay_threshold=0.0, delay_uniforms=None,
              episode=None, obs_out=None):
        o = self.ora.reset(customer_demand=customer_demand, noisy_delay=noisy_delay,
                           noisy_delay_threshold=noisy_delay_threshold, delay_uniforms=delay_uniforms)
        obs_out.copy_(torch.as_tensor(o))
        self.period, self.episode = 0, self.episode + 1
        return obs_out

    def step(self, actions, obs_out=None, reward_out=None, info=False, info_out=None):
        o, r, done, inf = self.ora.step(actions.numpy().astype(np.float64))
        obs_out.copy_(torch.as_tensor(o))
        reward_out.copy_(torch.as_tensor(np.asarray(r, dtype=np.float64)).reshape(reward_out.shape))
        if info_out is not None:
            for k in ("order", "demand", "acquisition", "ship", "profit"):
                info_out[k].copy_(torch.as_tensor(np.asarray(inf[k])).to(info_out[k].dtype))
        self.period += 1
        return obs_out, reward_out, done, info_out

    def close(self):
        pass


@pytest.fixture
def cpu_batch(monkeypatch):
    import imenv.rllib as rl
    monkeypatch.setattr(rl, "VectorInvEnv", OracleVectorEnv)
    return rl


def _inputs(meta, d):
    serial = meta["kind"] in ("IM", "MAIM")
    dem = d["customer_demand"][:, 0, :] if serial else d["customer_demand"]
    kw = dict(customer_demand=dem)
    if meta["noisy"]:
        kw.update(noisy_delay=True, noisy_delay_threshold=meta["noisy"], delay_uniforms=d["delay_uniforms"])
    return lambda episode: kw


@pytest.mark.parametrize("name", ["C1_IM4", "IM_div1", "IM4_noisy_delay"])
def test_vector_env_sequence(cpu_batch, name):
    meta, d = load_case(name)
    E, T = meta["E"], meta["T"]
    env = cpu_batch.InvVectorEnv(meta["kind"], meta["config"], num_envs=E, episode_inputs=_inputs(meta, d))
    assert env.num_envs == E and env.observation_space.shape == d["obs0"].shape[1:]
    assert env.get_unwrapped() == []
    for episode in range(2):
        obs = env.vector_reset() if episode == 0 else [env.reset_at(i) for i in range(E)]
        np.testing.assert_array_equal(np.stack(obs), d["obs0"])
        for t in range(T):
            obs, rew, dones, infos = env.vector_step([d["actions"][i, t] for i in range(E)])
            np.testing.assert_array_equal(np.stack(obs), d["obs"][:, t])
            np.testing.assert_array_equal(np.array(rew), d["reward"][:, t, 0])
            assert dones == [t == T - 1] * E and all(isinstance(r, float) for r in rew)
            for k in ("demand", "ship", "acquisition", "profit"):
                np.testing.assert_array_equal(np.stack([inf[k] for inf in infos]), d[k][:, t], err_msg=k)
            if t == 3:
                with pytest.raises(RuntimeError):
                    env.reset_at(1)
        with pytest.raises(RuntimeError):        # the batch's episode is over: step needs a reset first
            env.vector_step([d["actions"][i, 0] for i in range(E)])


@pytest.mark.parametrize("name", ["C2_MAIM4", "C4_MAIM_div1", "MAIM_div1_indep", "MAIM4_noisy_delay"])
def test_base_env_sequence(cpu_batch, name):
    meta, d = load_case(name)
    E, T = meta["E"], meta["T"]
    N = d["obs0"].shape[1]
    env = cpu_batch.InvMultiAgentBaseEnv(meta["kind"], meta["config"], num_envs=E, episode_inputs=_inputs(meta, d))
    ids = env.agent_ids
    obs, rew, dones, infos, off = env.poll()
    assert off == {} and sorted(obs) == list(range(E))
    for i in range(E):
        assert sorted(obs[i]) == sorted(ids)
        np.testing.assert_array_equal(np.stack([obs[i][ag] for ag in ids]), d["obs0"][i])
        assert rew[i] == {ag: None for ag in ids}
        assert dones[i] == dict({ag: False for ag in ids}, __all__=False) and infos[i] == {ag: {} for ag in ids}
    with pytest.raises(ValueError):              # lockstep: every env of the batch in one call
        env.send_actions({0: {ag: np.zeros(1) for ag in ids}})
    for episode in range(2):
        for t in range(T):
            env.send_actions({i: {ag: np.array([d["actions"][i, t, k]]) for k, ag in enumerate(ids)}
                              for i in range(E)})
            obs, rew, dones, infos, _ = env.poll()
            # the first poll after a try_reset also releases the reset's per-agent dones (RLlib's
            # _MultiAgentEnvState keeps them until an observation of the agent is released)
            want_done = dict({ag: False for ag in ids} if (episode and t == 0) else {}, __all__=t == T - 1)
            for i in range(E):
                assert dones[i] == want_done
                np.testing.assert_array_equal(np.stack([obs[i][ag] for ag in ids]), d["obs"][i, t])
                for k, ag in enumerate(ids):
                    assert rew[i][ag] == d["reward"][i, t, k if d["reward"].shape[-1] == N else 0]
                    inf = infos[i][ag]
                    assert inf["period"] == t + 1 and inf["actual order"] == d["order"][i, t, k]
                    assert inf["demand"] == d["demand"][i, t, k] and inf["profit"] == d["profit"][i, t, k]
        # after the episode: done envs refuse actions until try_reset; the first reset runs the batch's
        with pytest.raises(ValueError):
            env.send_actions({i: {ag: np.zeros(1) for ag in ids} for i in range(E)})
        for i in range(E):
            o = env.try_reset(i)
            np.testing.assert_array_equal(np.stack([o[ag] for ag in ids]), d["obs0"][i])
    env.stop()


def test_reset_rounds(cpu_batch):
    """A second whole round of resets at period 0 (every env reset again before any step) runs a new
    batched reset; a partial second round is refused."""
    meta, d = load_case("C1_IM4")
    E = meta["E"]
    env = cpu_batch.InvVectorEnv(meta["kind"], meta["config"], num_envs=E, episode_inputs=_inputs(meta, d))
    env.vector_reset()
    obs = [env.reset_at(i) for i in range(E)]          # a full new round
    np.testing.assert_array_equal(np.stack(obs), d["obs0"])
    assert env._b.episode == 1
    env.vector_step([d["actions"][i, 0] for i in range(E)])
    with pytest.raises(RuntimeError):
        env.reset_at(0)


@pytest.mark.parametrize("kind,cfg_name", [("IM", "C1_IM4"), ("MAIM_div", "C4_MAIM_div1")])
def test_oracle_episode_sequence_on_the_stand_in(cpu_batch, kind, cfg_name, monkeypatch):
    """tests/test_rllib_gpu.py's 64-env, two-episode oracle comparison, run here over the stand-in
    (the sequence and the shapes it feeds the oracle are checked on CPU before the GPU runs it)."""
    import test_rllib_gpu as g
    monkeypatch.setattr(g, "DEV", "cpu")
    g.test_batched_surfaces_match_the_oracle_over_episodes(kind, cfg_name)


@pytest.mark.parametrize("form", ["array1", "scalar", "list", "zero_d", "mixed"])
def test_send_actions_accepts_rllib_action_forms(cpu_batch, form):
    """An agent's action may come as a [1] array (Box(1) policies), a Python / NumPy scalar, a list or
    a 0-d array, and a batch may mix them: the stepped values are the same."""
    meta, d = load_case("C2_MAIM4")
    E = meta["E"]
    env = cpu_batch.InvMultiAgentBaseEnv(meta["kind"], meta["config"], num_envs=E, episode_inputs=_inputs(meta, d))
    ids = env.agent_ids
    env.poll()
    a = d["actions"][:, 0]
    conv = {"array1": lambda x, i: np.array([x]), "scalar": lambda x, i: float(x), "list": lambda x, i: [x],
            "zero_d": lambda x, i: np.array(x),
            "mixed": lambda x, i: (np.array([x]), np.float64(x), [x], np.array(x))[i % 4]}[form]
    env.send_actions({i: {ag: conv(a[i, k], i + k) for k, ag in enumerate(ids)} for i in range(E)})
    obs, rew, _, _, _ = env.poll()
    for i in range(E):
        np.testing.assert_array_equal(np.stack([obs[i][ag] for ag in ids]), d["obs"][i, 0])
    env.stop()


def test_infos_outlive_the_next_step(cpu_batch):
    """Infos handed out by one vector_step keep their values after the next one (RLlib stores them in its
    sample batches): every array in them is a copy, not a view of the host mirror the next step rewrites
    (IM_env.py:350 builds a fresh info dict per step)."""
    meta, d = load_case("C1_IM4")
    E = meta["E"]
    env = cpu_batch.InvVectorEnv(meta["kind"], meta["config"], num_envs=E, episode_inputs=_inputs(meta, d))
    env.vector_reset()
    _, _, _, infos0 = env.vector_step([d["actions"][i, 0] for i in range(E)])
    env.vector_step([d["actions"][i, 1] for i in range(E)])
    for k in ("demand", "ship", "acquisition", "profit"):
        np.testing.assert_array_equal(np.stack([inf[k] for inf in infos0]), d[k][:, 0], err_msg=k)
    ma_meta, md = load_case("C2_MAIM4")
    ma = cpu_batch.InvMultiAgentBaseEnv(ma_meta["kind"], ma_meta["config"], num_envs=ma_meta["E"],
                                        episode_inputs=_inputs(ma_meta, md))
    ids = ma.agent_ids
    ma.poll()
    ma.send_actions({i: {ag: np.array([md["actions"][i, 0, k]]) for k, ag in enumerate(ids)} for i in range(ma_meta["E"])})
    _, _, _, inf0, _ = ma.poll()
    ma.send_actions({i: {ag: np.array([md["actions"][i, 1, k]]) for k, ag in enumerate(ids)} for i in range(ma_meta["E"])})
    ma.poll()
    for i in range(ma_meta["E"]):
        for k, ag in enumerate(ids):
            assert inf0[i][ag]["profit"] == md["profit"][i, 0, k]


def test_second_poll_releases_nothing_new(cpu_batch):
    """A poll with no send_actions since the previous one hands out no observation again (RLlib's
    _MultiAgentEnvState releases an observation once)."""
    meta, d = load_case("C2_MAIM4")
    E = meta["E"]
    env = cpu_batch.InvMultiAgentBaseEnv(meta["kind"], meta["config"], num_envs=E, episode_inputs=_inputs(meta, d))
    ids = env.agent_ids
    env.poll()
    obs, _, _, _, _ = env.poll()
    assert all(obs[i] == {} for i in range(E))
    env.send_actions({i: {ag: np.array([d["actions"][i, 0, k]]) for k, ag in enumerate(ids)} for i in range(E)})
    obs, rew, _, _, _ = env.poll()
    assert all(sorted(obs[i]) == sorted(ids) for i in range(E))
    obs, rew, dones, _, _ = env.poll()
    assert all(obs[i] == {} and rew[i] == {} and dones[i] == {"__all__": False} for i in range(E))
    env.stop()

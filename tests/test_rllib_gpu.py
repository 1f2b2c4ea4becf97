"""The batched RLlib surfaces (imenv/rllib.py) against the reference: InvVectorEnv (RLlib VectorEnv,
single-agent classes) and InvMultiAgentBaseEnv (RLlib BaseEnv, multi-agent classes) drive the
reference's golden sessions (tests/golden, 32 envs x 30 periods each, made by importing the reference:
tools/gen_fixtures.py) bit for bit — observations, rewards, dones and every info field — through
RLlib's own call sequence (vector_reset / vector_step / reset_at; poll / send_actions / try_reset),
and 64 envs over two episodes against the oracle (oracle/im_oracle.py). Reference call sites:
inv_management.py:72-78 and MA_inv_management.py:83-84 (register_env), IM_env.py:287-360,
MAIM_env.py:330-411 (step results)."""
import numpy as np
import pytest

from golden_io import case_names, load_case

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SINGLE = [c for c in case_names() if load_case(c)[0]["kind"] in ("IM", "IM_div")]
MULTI = [c for c in case_names() if load_case(c)[0]["kind"] in ("MAIM", "MAIM_div")]


def _inputs(meta, d):
    serial = meta["kind"] in ("IM", "MAIM")
    dem = d["customer_demand"][:, 0, :] if serial else d["customer_demand"]
    kw = dict(customer_demand=dem)
    if meta["noisy"]:
        kw.update(noisy_delay=True, noisy_delay_threshold=meta["noisy"], delay_uniforms=d["delay_uniforms"])
    return lambda episode: kw


@pytest.mark.parametrize("name", SINGLE)
def test_vector_env_replays_golden_sessions(name):
    from imenv.rllib import InvVectorEnv
    meta, d = load_case(name)
    E, T = meta["E"], meta["T"]
    env = InvVectorEnv(meta["kind"], meta["config"], num_envs=E, device=DEV, episode_inputs=_inputs(meta, d))
    assert env.num_envs == E and env.observation_space.shape == d["obs0"].shape[1:]
    for episode in range(2):
        if episode == 0:
            obs = env.vector_reset()
        else:       # RLlib resets each done env (the first call runs the batch's reset)
            obs = [env.reset_at(i) for i in range(E)]
        np.testing.assert_array_equal(np.stack(obs), d["obs0"])
        for t in range(T):
            acts = [d["actions"][i, t] for i in range(E)]
            obs, rew, dones, infos = env.vector_step(acts)
            np.testing.assert_array_equal(np.stack(obs), d["obs"][:, t])
            np.testing.assert_array_equal(np.array(rew), d["reward"][:, t, 0])
            assert dones == [t == T - 1] * E
            for k in ("demand", "ship", "acquisition", "profit"):
                np.testing.assert_array_equal(np.stack([inf[k] for inf in infos]), d[k][:, t], err_msg=k)
            assert all(inf["period"] == t for inf in infos)
            if t == 5 and episode == 0:
                with pytest.raises(RuntimeError):
                    env.reset_at(3)         # lockstep: no reset in the middle of the batch's episode
    env.close()


@pytest.mark.parametrize("name", MULTI)
def test_multi_agent_base_env_replays_golden_sessions(name):
    from imenv.rllib import InvMultiAgentBaseEnv
    meta, d = load_case(name)
    E, T = meta["E"], meta["T"]
    N = d["obs0"].shape[1]
    env = InvMultiAgentBaseEnv(meta["kind"], meta["config"], num_envs=E, device=DEV,
                               episode_inputs=_inputs(meta, d))
    ids = env.agent_ids
    assert ids == [("stage_" if meta["kind"] == "MAIM" else "node_") + str(k) for k in range(N)]
    obs, rew, dones, infos, off = env.poll()
    assert off == {} and sorted(obs) == list(range(E))
    for i in range(E):
        for k, ag in enumerate(ids):
            np.testing.assert_array_equal(obs[i][ag], d["obs0"][i, k])
        assert rew[i] == {ag: None for ag in ids} and dones[i] == {ag: False for ag in ids} | {"__all__": False}
        assert infos[i] == {ag: {} for ag in ids}
    for episode in range(2):
        for t in range(T):
            env.send_actions({i: {ag: np.array([d["actions"][i, t, k]]) for k, ag in enumerate(ids)}
                              for i in range(E)})
            obs, rew, dones, infos, _ = env.poll()
            last = t == T - 1
            for i in range(E):
                assert dones[i]["__all__"] == last
                for k, ag in enumerate(ids):
                    np.testing.assert_array_equal(obs[i][ag], d["obs"][i, t, k])
                    want_r = d["reward"][i, t, k if d["reward"].shape[-1] == N else 0]
                    assert rew[i][ag] == want_r, (i, t, ag)
                    inf = infos[i][ag]
                    assert inf["period"] == t + 1
                    for key, src in (("demand", "demand"), ("ship", "ship"), ("acquisition", "acquisition"),
                                     ("actual order", "order"), ("profit", "profit")):
                        assert inf[key] == d[src][i, t, k], (key, i, t, ag)
        with pytest.raises(ValueError):          # a done env takes no more actions until it is reset
            env.send_actions({i: {ag: np.zeros(1) for ag in ids} for i in range(E)})
        for i in range(E):
            o = env.try_reset(i)
            for k, ag in enumerate(ids):
                np.testing.assert_array_equal(o[ag], d["obs0"][i, k])
    env.stop()


@pytest.mark.parametrize("kind,cfg_name", [("IM", "C1_IM4"), ("MAIM", "C2_MAIM4"), ("IM_div", "IM_div1"),
                                           ("MAIM_div", "C4_MAIM_div1")])
def test_batched_surfaces_match_the_oracle_over_episodes(kind, cfg_name):
    """64 envs, two episodes of fresh host demand and actions each: every env equals the oracle."""
    from imenv.rllib import InvMultiAgentBaseEnv, InvVectorEnv
    from oracle.im_oracle import OracleEnv
    meta, _ = load_case(cfg_name)
    cfg = meta["config"]
    E = 64
    rs = np.random.RandomState(7)
    ora = OracleEnv(kind, cfg, n_envs=E)
    N, T, R = ora.N, ora.num_periods, len(ora.retailers)
    serial = kind in ("IM", "MAIM")
    demands = [rs.poisson(5, (E, T) if serial else (E, R, T)) for _ in range(2)]
    acts = [rs.uniform(-1, 1, (T, E, N)) for _ in range(2)]
    inputs = lambda ep: dict(customer_demand=demands[ep])
    ma = kind in ("MAIM", "MAIM_div")
    env = (InvMultiAgentBaseEnv if ma else InvVectorEnv)(kind, cfg, num_envs=E, device=DEV, episode_inputs=inputs)
    for ep in range(2):
        o_ref = ora.reset(customer_demand=demands[ep])
        if ma:
            if ep == 0:
                obs = env.poll()[0]
            else:
                obs = {i: env.try_reset(i) for i in range(E)}
            got = np.stack([np.stack([obs[i][ag] for ag in env.agent_ids]) for i in range(E)])
        else:
            got = np.stack(env.vector_reset() if ep == 0 else [env.reset_at(i) for i in range(E)])
        np.testing.assert_array_equal(got, o_ref)
        for t in range(T):
            o_ref, r_ref, _, _ = ora.step(acts[ep][t])
            if ma:
                env.send_actions({i: {ag: acts[ep][t, i, k:k + 1] for k, ag in enumerate(env.agent_ids)}
                                  for i in range(E)})
                obs, rew, _, _, _ = env.poll()
                got = np.stack([np.stack([obs[i][ag] for ag in env.agent_ids]) for i in range(E)])
                got_r = np.array([[rew[i][ag] for ag in env.agent_ids] for i in range(E)])
                r_ref = np.asarray(r_ref)
                r_ref = r_ref if r_ref.ndim == 2 else np.repeat(r_ref[:, None], N, axis=1)
            else:
                obs, rew, _, _ = env.vector_step(list(acts[ep][t]))
                got, got_r = np.stack(obs), np.array(rew)
            np.testing.assert_array_equal(got, o_ref)
            np.testing.assert_array_equal(got_r, r_ref)
    (env.stop if ma else env.close)()


def test_surfaces_refuse_the_other_kind():
    from imenv.rllib import InvMultiAgentBaseEnv, InvVectorEnv
    meta, _ = load_case("C2_MAIM4")
    with pytest.raises(ValueError):
        InvVectorEnv("MAIM", meta["config"], num_envs=4, device=DEV)
    with pytest.raises(ValueError):
        InvMultiAgentBaseEnv("IM", meta["config"], num_envs=4, device=DEV)

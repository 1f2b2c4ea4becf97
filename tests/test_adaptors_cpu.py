"""Host-side checks of the drop-in adaptors that need no GPU."""
import numpy as np
import pytest
import torch


def test_rescale_rev_scale_match_reference_formulas():
    from imenv.envs import rescale, rev_scale
    v = np.arange(0, 31, dtype=np.float64)
    # IM_env.py:435-456
    np.testing.assert_array_equal(rescale(v, 0, 30, -1, 1), -1 + ((v - 0) * (1 - -1)) / (30 - 0))
    x = np.linspace(-1, 1, 9)
    np.testing.assert_array_equal(rev_scale(x, 0, 30, -1, 1), ((x - -1) * (30 - 0)) / (1 - -1) + 0)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
def test_adaptor_fails_loudly_without_gpu():
    from imenv import ImEnvNativeError
    from imenv.envs import MultiAgentInvManagement
    cfg = dict(num_stages=3, num_periods=5, demand_dist="poisson", mu=5)
    with pytest.raises(ImEnvNativeError):
        MultiAgentInvManagement(cfg)
    # the reference's constructor pops its keys from the caller's dict before it fails
    assert cfg == {"mu": 5}


def test_box_space_fields():
    from imenv.spaces import Box
    b = Box(low=np.ones(3) * -1, high=np.ones(3), dtype=np.float64, shape=(3,))
    assert b.shape == (3,) and b.dtype == np.float64
    assert b.contains(b.sample())

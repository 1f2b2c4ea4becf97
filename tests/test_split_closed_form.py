"""The two-child round robin of the divergent split in closed form (csrc/imenv_device.h rr_closed<2>,
restated statement by statement in tools/check_rr_closed.py) equals the reference's literal loop
(IM_div_env.py:413-498) on every small case, guard trips included. The kernels themselves are pinned
against the reference on trees by tests/test_gpu_parity.py and tests/test_fuzz_gpu.py."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

from check_rr_closed import check  # noqa: E402


def test_two_child_round_robin_closed_form_equals_literal_loop():
    n, bad = check(xr=range(-3, 11), ar=range(-2, 25), lims=(0, 1, 2, 4, 7, 60))
    assert n > 50000
    assert not bad, bad[:5]

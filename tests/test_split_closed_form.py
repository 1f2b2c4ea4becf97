"""Closed forms of the step kernel checked against the reference's own expressions on CPU: the two-child
round robin of the divergent split (csrc/imenv_device.h rr_closed<2>, restated in tools/check_rr_closed.py)
against the literal loop (IM_div_env.py:413-498), guard trips included. The kernels themselves are
pinned against the reference by tests/test_gpu_parity.py and tests/test_fuzz_gpu.py."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

from check_rr_closed import check  # noqa: E402


def test_two_child_round_robin_closed_form_equals_literal_loop():
    n, bad = check(xr=range(-3, 11), ar=range(-2, 25), lims=(0, 1, 2, 4, 7, 60))
    assert n > 50000
    assert not bad, bad[:5]


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



def test_closed_form_at_the_largest_accepted_guard_limit():
    """imenv_create accepts split guard limits up to 2^30 (tools/asan_host_check.py: 2^30 + 1 and
    INT32_MAX are refused): at 2^30 the int32 closed form still equals the literal loop, while at
    INT32_MAX its `lim + 1` would wrap (the reason for the bound)."""
    n, bad = check(xr=range(-2, 9), ar=range(-2, 20), lims=(1 << 30,))
    assert n > 4000 and not bad, bad[:5]
    _, bad = check(xr=range(1, 4), ar=range(1, 6), lims=(2 ** 31 - 1,))
    assert bad      # documents the overflow that validation prevents

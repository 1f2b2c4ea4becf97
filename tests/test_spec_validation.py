"""The C ABI's error contract on malformed specs (CPU, no GPU): every spec the reference's
constructors would refuse, and every value this build cannot represent, comes back from
imenv_jit_check / imenv_create as IMENV_E_INVALID / IMENV_E_UNSUPPORTED with a message, before any
device call (reference: IM_env.py:203-207, MAIM_env.py:158-171). The same cases run under
AddressSanitizer + UndefinedBehaviorSanitizer in tools/asan_host_check.py (profiles/r03/asan)."""
import ctypes
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _lib():
    from imenv import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libimenv.so not built")
    return _native, _native.load()


@pytest.mark.parametrize("base_cfg", ["C2", "C4"])
def test_malformed_specs_are_rejected(base_cfg):
    import asan_host_check as ahc
    import bench
    from imenv import build_spec
    nat, lib = _lib()
    kind, cfg = bench.CONFIGS[base_cfg][:2]
    base = build_spec(kind, cfg).to_c()
    log = ctypes.create_string_buffer(4096)
    cases = ahc.malformed(base)
    assert len(cases) >= 50
    for name, spec in cases:
        rc = lib.imenv_jit_check(ctypes.byref(spec), b"gfx-invalid-arch", 0, log, len(log))
        assert rc in (nat.E_INVALID, nat.E_UNSUPPORTED), (name, rc)
        assert "hipRTC" not in lib.imenv_last_error().decode(), name     # refused by validation itself
        h = ctypes.c_void_p()
        rc = lib.imenv_create(ctypes.byref(spec), 16, 0, 0, ctypes.byref(h))
        assert rc in (nat.E_INVALID, nat.E_UNSUPPORTED) and not h.value, (name, rc)
        assert lib.imenv_last_error().decode(), name


@pytest.mark.parametrize("base_cfg", ["C2", "C4"])
def test_odd_but_valid_specs_validate(base_cfg):
    """Zero capacities as observation denominators and NaN noise thresholds are accepted (the
    reference runs with them): imenv_create validates them and then stops at its first device call
    here (no GPU: IMENV_E_HIP), or succeeds on a GPU box."""
    import asan_host_check as ahc
    import bench
    from imenv import build_spec
    nat, lib = _lib()
    kind, cfg = bench.CONFIGS[base_cfg][:2]
    base = build_spec(kind, cfg).to_c()
    for name, spec in ahc.odd_but_valid(base) + [("base", base)]:
        h = ctypes.c_void_p()
        rc = lib.imenv_create(ctypes.byref(spec), 16, 0, 0, ctypes.byref(h))
        assert rc in (0, nat.E_HIP), (name, rc, lib.imenv_last_error())
        if h.value:
            lib.imenv_destroy(h)

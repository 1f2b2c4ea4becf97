"""CPU checks of the drop-in boundary: libimenv.so loads (no GPU needed), exports every entry
point include/imenv.h declares, and the ctypes ImEnvSpec layout matches the compiled one."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "imenv.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(imenv_[a-z_]+)\s*\(", src)))


def test_header_declares_the_abi():
    names = declared_functions()
    for must in ("imenv_create", "imenv_reset", "imenv_step", "imenv_get_state", "imenv_destroy",
                 "imenv_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from imenv import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libimenv.so not built (python __graft_entry__.py build)")
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    bound = {name for name, _, _ in _native.SYMBOLS}
    assert bound == set(declared_functions()), set(declared_functions()) ^ bound


def test_abi_version_and_spec_layout():
    from imenv import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libimenv.so not built")
    lib = _native.load()
    assert lib.imenv_abi_version() == _native.ABI_VERSION
    assert lib.imenv_spec_size() == ctypes.sizeof(_native.ImEnvSpec)


def test_missing_library_fails_loudly(tmp_path):
    from imenv import _native
    with pytest.raises(_native.ImEnvNativeError):
        _native.load(str(tmp_path / "nope.so"))


def test_jit_specialiser_compiles_every_golden_spec():
    """hipRTC builds the spec-specialised step kernel for every golden config (no device needed),
    for the bench's call flags (f32 actions/obs, in-kernel draws) and the parity-test flags
    (f64 actions/obs, per-env demand table, host-fed delay uniforms, harness metrics)."""
    from golden_io import case_names, load_case
    from imenv import _native, build_spec
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libimenv.so not built")
    lib = _native.load()
    log = ctypes.create_string_buffer(1 << 16)
    for name in case_names():
        meta, _ = load_case(name)
        spec = build_spec(meta["kind"], meta["config"]).to_c()
        sets = [0, 1 | 2 | (_native.LAYOUT_PER_ENV << 5) | (16 if meta["noisy"] else 0) | 1024]
        if name in ("C2_MAIM4", "C3_IM8", "C4_MAIM_div1", "MAIM_div2_share", "IM4_td_pd_pa_L2"):
            sets += [2048, 2 | 2048]          # streaming stores (IMENV_STORE_STREAM), f32 and f64 obs
        # small launches (64-env blocks; uint8 specs of <= 8 nodes take the 16/32-byte state records),
        # write-through obs and state stores as the default policy picks them there, and a tree's
        # compact backlog_to rows, with f32 and f64 observations
        sets += [8192 | 16384 | 32768, 2 | 8192 | 16384 | 32768, 1 | 2 | (_native.LAYOUT_PER_ENV << 5) | 32768,
                 8192 | 16384 | 32768 | 65536 | 131072, 2 | 8192 | 65536 | 131072,   # slim: no info, whole blocks
                 8192 | 16384 | 32768 | 65536 | 131072 | 262144, 2 | 8192 | 65536 | 131072 | 262144]   # + aligned
        for flags in sets:
            rc = lib.imenv_jit_check(ctypes.byref(spec), b"gfx950", flags, log, len(log))
            assert rc == 0, (name, flags, log.value.decode()[:2000])


def test_jit_rollout_kernel_compiles_for_scalar_reward_specs():
    """hipRTC builds the fused base-stock rollout kernel (rollout_body) for every golden spec with a
    scalar reward: host demand table + objective (one replay per retailer row for > 1 retailer),
    and in-kernel draws + noisy delay (+ noisy demand for the tree specs)."""
    from golden_io import case_names, load_case
    from imenv import _native, build_spec
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libimenv.so not built")
    lib = _native.load()
    log = ctypes.create_string_buffer(1 << 16)
    for name in case_names():
        meta, _ = load_case(name)
        hs = build_spec(meta["kind"], meta["config"])
        if hs.reward_mode == _native.REWARD_INDEPENDENT:
            continue
        spec = hs.to_c()
        nd = 4 if hs.noisy_demand else 0
        for rk in (1 | 8, 2 | nd | 8):
            flags = (1 << 12) | (rk << 13)
            rc = lib.imenv_jit_check(ctypes.byref(spec), b"gfx950", flags, log, len(log))
            assert rc == 0, (name, rk, log.value.decode()[:2000])


def test_jit_plan_rollout_kernel_compiles():
    """hipRTC builds the plan-replay form of the rollout kernel (ACT = shared / per-episode plan,
    float32 and float64 plans) for the golden plan-replay specs and the bench's C2 spec."""
    from golden_io import load_base_stock
    from imenv import _native, build_spec
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libimenv.so not built")
    lib = _native.load()
    log = ctypes.create_string_buffer(1 << 16)
    meta, _ = load_base_stock("plan_replay.npz")
    for name, m in sorted(meta.items()):
        spec = build_spec(m["kind"], m["config"]).to_c()
        for rk in (1 | (1 << 4) | 64, 1 | (2 << 4), 2 | (2 << 4) | 64):
            flags = (1 << 12) | (rk << 13)
            rc = lib.imenv_jit_check(ctypes.byref(spec), b"gfx950", flags, log, len(log))
            assert rc == 0, (name, rk, log.value.decode()[:2000])
    # a plan rollout with an objective is not a kernel
    spec = build_spec(meta["SHLP4"]["kind"], meta["SHLP4"]["config"]).to_c()
    assert lib.imenv_jit_check(ctypes.byref(spec), b"gfx950", (1 << 12) | ((8 | (2 << 4)) << 13), log, len(log)) != 0


def test_library_embeds_the_current_device_sources():
    """The hipRTC specialiser compiles the step kernel from device sources embedded in libimenv.so at
    build time (imenv_rtc_src.inc, generated by __graft_entry__.build(), not tracked). A stale library
    would ship a different kernel body than the one the tests and the oracle were checked against, so
    the embedded text must equal imenv_device.h and imenv.h byte for byte."""
    from imenv import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libimenv.so not built")
    blob = open(_native.LIB_PATH, "rb").read()
    for path in (os.path.join(ROOT, "marl-for-im_amd", "csrc", "imenv_device.h"), HEADER):
        text = open(path, "rb").read()
        assert blob.find(text + b"\0") >= 0, \
            "%s differs from the copy embedded in libimenv.so: rebuild (python __graft_entry__.py build)" % path


def _dump_jit_source(cname, tmp_path, extra_env=None):
    """The generated hipRTC source of a bench config's step kernel (f32 actions / obs, write-through
    stores), from a fresh process (IMENV_JIT_DUMP; the compile cache is per process)."""
    import subprocess
    import sys
    code = ("import ctypes, bench; from imenv import _native, build_spec; lib = _native.load(); "
            "k, c = bench.CONFIGS[%r][:2]; s = build_spec(k, c).to_c(); log = ctypes.create_string_buffer(65536); "
            "rc = lib.imenv_jit_check(ctypes.byref(s), b'gfx950', 0x2000, log, len(log)); "
            "assert rc == 0, log.value.decode()[:2000]" % cname)
    os.makedirs(tmp_path, exist_ok=True)
    env = dict(os.environ, IMENV_JIT_DUMP=str(tmp_path), **(extra_env or {}))
    env["PYTHONPATH"] = os.pathsep.join([ROOT, os.path.join(ROOT, "marl-for-im_amd")])
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    srcs = [p for p in os.listdir(tmp_path) if p.endswith(".hip")]
    assert len(srcs) == 1, srcs
    return open(os.path.join(tmp_path, srcs[0])).read()


@pytest.mark.parametrize("cname", ["C2", "C3", "C4"])
def test_bench_kernels_use_unguarded_verified_observations(cname, tmp_path):
    """Every scaled observation value of the bench configs is emitted as a closed form verified
    exhaustively over [0, vbound] with no per-value range guard: the values an observation reads are
    state values, bounded by vbound (imenv_capi.hip state_bound: capacities, capped backlog, demand and
    shipment bounds), and that whole range is verified (imenv_jit.hip emit_obs_hooks keeps the guard
    when it cannot verify all of it)."""
    from imenv import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libimenv.so not built")
    src = _dump_jit_source(cname, tmp_path)
    assert "if ((unsigned)v <=" not in src
    assert "imenv_step_jit_wt(" in src


def test_extra_jit_options_rename_the_kernel(tmp_path):
    """IMENV_JIT_OPTS experiments get a kernel name of their own (a hash of the options), so a trace or
    PMC summary of an experiment never matches the production kernel; diagnostic switches are named
    _diag_ (and refused at kernel load unless IMENV_DIAG=1: tests/test_jit_gpu.py)."""
    from imenv import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libimenv.so not built")
    src = _dump_jit_source("C2", tmp_path / "opt", {"IMENV_JIT_OPTS": "-DIMENV_SLAB_BATCH=1"})
    assert re.search(r"imenv_step_jit_wt_opt_[0-9a-f]{8}\(", src)
    src = _dump_jit_source("C2", tmp_path / "diag", {"IMENV_JIT_OPTS": "-DIMENV_ABLATE=16"})
    assert re.search(r"imenv_step_jit_wt_diag_[0-9a-f]{8}\(", src)

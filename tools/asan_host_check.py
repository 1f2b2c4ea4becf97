#!/usr/bin/env python3
"""AddressSanitizer + UndefinedBehaviorSanitizer run of libimenv's HOST code (no GPU needed).

    python tools/asan_host_check.py [--out DIR] [--rebuild]

1. Builds every libimenv source with the sanitizers on the host side only (`-Xarch_host
   -fsanitize=...`; device code is compiled as usual) and links tools/asan/asan_driver.cpp against
   the objects (tools/bin/asan/asan_driver).
2. Writes the spec records the driver reads: every golden configuration of tests/golden (the four
   reference classes, every observation-flag combination, 24 drawn configurations), the bench
   configurations C2 / C3 / C4 and the plan-replay / base-stock configurations, each expected to
   validate; plus malformed specs derived from them (out-of-range node / period / feature counts,
   delays, children and parents, prev_length, history and transit indices, modes, non-finite
   prices / costs / scaling, Poisson means, uniform bounds), each expected to be rejected with
   IMENV_E_INVALID / IMENV_E_UNSUPPORTED (the reference raises at __init__: IM_env.py:203-207,
   MAIM_env.py:158-171).
3. Runs the driver: spec validation and derivation, observation tables, the hipRTC source
   generator (and a real gfx950 compile for a subset), imenv_create up to its first device call,
   and the argument checks of every entry point. Any sanitizer report or wrong status fails.
Results go to DIR/summary.json (default profiles/r03/asan).
"""
import ctypes
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-for-im_amd"), os.path.join(ROOT, "tests")]

import __graft_entry__ as ge  # noqa: E402

BIN = os.path.join(ROOT, "tools", "bin", "asan")
DRIVER_SRC = os.path.join(ROOT, "tools", "asan", "asan_driver.cpp")
DRIVER = os.path.join(BIN, "asan_driver")
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
       "-Xarch_host", "-fno-sanitize-recover=all", "-Xarch_host", "-fno-omit-frame-pointer"]


def build(rebuild=False):
    os.makedirs(BIN, exist_ok=True)
    inc = ge._write_rtc_inc()
    flags = [f for f in ge.HIPFLAGS if f != "-O3"] + ["-O1", "-g"]
    objs, procs = [], []
    for src in ge.SRCS:
        obj = os.path.join(BIN, os.path.basename(src) + ".o")
        objs.append(obj)
        if rebuild or ge._stale(obj, [src, inc] + ge.HDRS):
            cmd = [ge.HIPCC] + flags + SAN + ["-I", os.path.join(ROOT, "include"), "-I", ge.GEN, "-c", "-o", obj, src]
            procs.append(subprocess.Popen(cmd))
    if any(p.wait() != 0 for p in procs):
        raise SystemExit("sanitized compile failed")
    if rebuild or procs or ge._stale(DRIVER, objs + [DRIVER_SRC]):
        dobj = os.path.join(BIN, "asan_driver.o")     # plain C++ over the C ABI: host compiler only
        subprocess.check_call([os.path.join(os.path.dirname(os.path.realpath(ge.HIPCC)), "..", "lib", "llvm", "bin",
                                            "clang++"), "-c", "-O1", "-g", "-std=c++17", "-fsanitize=address",
                               "-fsanitize=undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
                               "-I", os.path.join(ROOT, "include"), "-o", dobj, DRIVER_SRC])
        subprocess.check_call([ge.HIPCC, "--offload-arch=gfx950", "-fsanitize=address", "-fsanitize=undefined",
                               "-fno-gpu-sanitize", "-o", DRIVER, dobj] + objs + ["-lhiprtc"])


def good_specs():
    """(name, ImEnvSpec, jit) for every configuration the tests pin."""
    import bench
    from golden_io import case_names, fuzz_case_names, load_case, load_base_stock
    from imenv import build_spec
    out = []
    for name in case_names():
        meta, _ = load_case(name)
        out.append((name, build_spec(meta["kind"], meta["config"]).to_c(), False))
    for name in fuzz_case_names():
        meta, _ = load_case(name)
        out.append((name, build_spec(meta["kind"], meta["config"]).to_c(), False))
    for key in ("plan_replay.npz", "base_stock.npz"):
        try:
            meta, _ = load_base_stock(key)
        except Exception:
            continue
        for name, m in sorted(meta.items()):
            out.append((key[:-4] + "/" + name, build_spec(m["kind"], m["config"]).to_c(), False))
    for c in ("C2", "C3", "C4"):     # the bench configurations: compiled for gfx950 for real
        kind, cfg = bench.CONFIGS[c][:2]
        out.append(("bench_" + c, build_spec(kind, cfg).to_c(), True))
    return out


def malformed(base):
    """(name, spec) variants of a valid spec that the ABI must reject."""
    from imenv import _native as nat
    N = base.num_nodes

    def mut(name, fn):
        s = type(base)()
        ctypes.memmove(ctypes.byref(s), ctypes.byref(base), ctypes.sizeof(base))
        fn(s)
        return (name, s)

    nan, inf = float("nan"), float("inf")
    v = [
        mut("abi_version", lambda s: setattr(s, "abi_version", 99)),
        mut("num_nodes_0", lambda s: setattr(s, "num_nodes", 0)),
        mut("num_nodes_neg", lambda s: setattr(s, "num_nodes", -3)),
        mut("num_nodes_17", lambda s: setattr(s, "num_nodes", 17)),
        mut("num_periods_0", lambda s: setattr(s, "num_periods", 0)),
        mut("num_periods_huge", lambda s: setattr(s, "num_periods", 100001)),
        mut("delay_0", lambda s: s.delay.__setitem__(1, 0)),
        mut("delay_neg", lambda s: s.delay.__setitem__(0, -2)),
        mut("delay_65", lambda s: s.delay.__setitem__(N - 1, 65)),
        mut("parent_out_of_range", lambda s: s.parent.__setitem__(1, 40)),
        mut("parent_self", lambda s: s.parent.__setitem__(1, 1)),
        mut("two_factories", lambda s: [s.parent.__setitem__(i, -1) for i in range(N)]),
        mut("children_9", lambda s: s.num_children.__setitem__(0, 9)),
        mut("children_neg", lambda s: s.num_children.__setitem__(0, -1)),
        mut("child_out_of_range", lambda s: (s.num_children.__setitem__(0, 1), s.children[0].__setitem__(0, 99))),
        mut("retailer_slot_range", lambda s: [s.retailer_slot.__setitem__(i, 7) for i in range(N)
                                              if s.retailer_slot[i] >= 0]),
        mut("num_retailers_0", lambda s: setattr(s, "num_retailers", 0)),
        mut("num_retailers_mismatch", lambda s: setattr(s, "num_retailers", s.num_retailers + 1)),
        mut("demand_parent_range", lambda s: s.demand_parent.__setitem__(0, 16)),
        mut("num_features_0", lambda s: setattr(s, "num_features", 0)),
        mut("num_features_65", lambda s: setattr(s, "num_features", 65)),
        mut("prev_length_0", lambda s: setattr(s, "prev_length", 0)),
        mut("prev_length_9", lambda s: setattr(s, "prev_length", 9)),
        mut("feat_group_8", lambda s: s.feat_group.__setitem__(0, 8)),
        mut("feat_group_neg", lambda s: s.feat_group.__setitem__(0, -1)),
        mut("feat_index_neg", lambda s: s.feat_index.__setitem__(0, -1)),
        mut("hist_index_ge_L", lambda s: (s.feat_group.__setitem__(0, nat.G_DEMAND_HIST if hasattr(nat, "G_DEMAND_HIST") else 3),
                                           s.feat_index.__setitem__(0, s.prev_length))),
        mut("transit_index_ge_dmax", lambda s: (s.feat_group.__setitem__(0, 5), s.feat_index.__setitem__(0, 64))),
        mut("group_mode_4", lambda s: s.group_mode.__setitem__(0, 4)),
        mut("decode_mode_5", lambda s: setattr(s, "decode_mode", 5)),
        mut("reward_mode_3", lambda s: setattr(s, "reward_mode", 3)),
        mut("a_eq_b", lambda s: (setattr(s, "standardise_actions", 1), setattr(s, "a", 1.0), setattr(s, "b", 1.0))),
        mut("a_nan", lambda s: (setattr(s, "standardise_actions", 1), setattr(s, "a", nan))),
        mut("b_inf", lambda s: (setattr(s, "standardise_actions", 1), setattr(s, "b", inf))),
        mut("poisson_mu_0", lambda s: (setattr(s, "demand_dist", 2), setattr(s, "poisson_mu", 0.0))),
        mut("poisson_mu_nan", lambda s: (setattr(s, "demand_dist", 2), setattr(s, "poisson_mu", nan))),
        mut("poisson_mu_neg", lambda s: (setattr(s, "demand_dist", 2), setattr(s, "poisson_mu", -5.0))),
        mut("poisson_mu_huge", lambda s: (setattr(s, "demand_dist", 2), setattr(s, "poisson_mu", 1e6))),
        mut("poisson_mu_inf", lambda s: (setattr(s, "demand_dist", 2), setattr(s, "poisson_mu", inf))),
        mut("uniform_low_ge_high", lambda s: (setattr(s, "demand_dist", 3), setattr(s, "uniform_low", 5),
                                              setattr(s, "uniform_high", 5))),
        mut("demand_dist_9", lambda s: setattr(s, "demand_dist", 9)),
        mut("inv_max_neg", lambda s: s.inv_max.__setitem__(0, -1)),
        mut("order_max_neg", lambda s: s.order_max.__setitem__(0, -1)),
        mut("init_inv_neg", lambda s: s.init_inv.__setitem__(0, -1)),
        mut("sell_price_nan", lambda s: s.sell_price.__setitem__(0, nan)),
        mut("buy_price_inf", lambda s: s.buy_price.__setitem__(N - 1, -inf)),
        mut("stock_cost_nan", lambda s: s.stock_cost.__setitem__(0, nan)),
        mut("backlog_cost_inf", lambda s: s.backlog_cost.__setitem__(0, inf)),
        mut("inv_target_nan", lambda s: s.inv_target.__setitem__(0, nan)),
        mut("group_den_nan", lambda s: s.group_den[0].__setitem__(0, nan)),
        mut("group_clip_neg_inf", lambda s: (s.group_mode.__setitem__(5, 3), s.group_clip[5].__setitem__(0, -inf))),
        mut("split_limit_neg", lambda s: s.split_limit[0].__setitem__(0, -1)),
        # the closed-form split counts rounds up to limit + 1 in int32: limits past 2^30 are refused
        mut("split_limit_int32_max", lambda s: s.split_limit[0].__setitem__(1, 2147483647)),
        mut("split_limit_2p30_plus_1", lambda s: s.split_limit[0].__setitem__(2, (1 << 30) + 1)),
    ]
    return v


def odd_but_valid(base):
    """Specs the reference accepts with odd values (zero capacities as observation denominators, NaN
    noise thresholds: `uniform() < nan` is never true): they must validate without undefined behaviour."""
    def mut(name, fn):
        s = type(base)()
        ctypes.memmove(ctypes.byref(s), ctypes.byref(base), ctypes.sizeof(base))
        fn(s)
        return (name, s)
    nan = float("nan")
    return [
        mut("group_den_0", lambda s: s.group_den[0].__setitem__(0, 0.0)),
        mut("noisy_delay_thr_nan", lambda s: (setattr(s, "noisy_delay", 1), setattr(s, "noisy_delay_threshold", nan))),
        mut("noisy_demand_thr_nan", lambda s: (setattr(s, "noisy_demand", 1), setattr(s, "noisy_demand_threshold", nan))),
        mut("inv_max_0", lambda s: (s.inv_max.__setitem__(0, 0), s.order_max.__setitem__(0, 0))),
    ]


def write_records(path, records):
    with open(path, "wb") as f:
        for name, spec, expect, jit in records:
            f.write(int(expect).to_bytes(4, "little", signed=True))
            f.write(int(jit).to_bytes(4, "little", signed=True))
            f.write(name.encode()[:63].ljust(64, b"\0"))
            f.write(bytes(spec))


def main():
    out = os.path.join(ROOT, "profiles", "r03", "asan")
    if "--out" in sys.argv:
        out = sys.argv[sys.argv.index("--out") + 1]
    os.makedirs(out, exist_ok=True)
    t0 = time.time()
    build(rebuild="--rebuild" in sys.argv)
    t_build = time.time() - t0
    good = good_specs()
    records = [(n, s, 0, j) for n, s, j in good]
    bad = []
    for base_name in ("bench_C2", "bench_C4"):
        base = next(s for n, s, _ in good if n == base_name)
        bad += [(base_name + ":" + n, s, 1, 0) for n, s in malformed(base)]
        records += [(base_name + ":" + n, s, 0, 0) for n, s in odd_but_valid(base)]
    records += bad
    specs = os.path.join(out, "specs.bin")
    write_records(specs, records)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1:detect_odr_violation=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", HIP_VISIBLE_DEVICES=os.environ.get(
                   "HIP_VISIBLE_DEVICES", ""),
               LSAN_OPTIONS="suppressions=" + os.path.join(ROOT, "tools", "asan", "lsan.supp"))
    t1 = time.time()
    r = subprocess.run([DRIVER, specs], capture_output=True, text=True, env=env, timeout=1800)
    res = {"driver": os.path.relpath(DRIVER, ROOT), "returncode": r.returncode, "build_s": round(t_build, 1),
           "run_s": round(time.time() - t1, 1), "records": len(records), "valid": sum(1 for r in records if r[2] == 0), "malformed": len(bad),
           "sanitizers": "address,undefined (host code; -fno-sanitize-recover=all)",
           "stdout": r.stdout[-2000:], "stderr_tail": r.stderr[-6000:]}
    try:
        res.update(json.loads(r.stdout.strip().splitlines()[-1]))
    except Exception:
        pass
    os.remove(specs)
    with open(os.path.join(out, "summary.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("stdout", "stderr_tail")}))
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-6000:])
        raise SystemExit(1)


if __name__ == "__main__":
    main()

"""ctypes binding of include/imenv.h (libimenv.so, built in-tree for gfx950).

The HIP library IS the product: there is no CPU fallback. ``load()`` raises
ImEnvNativeError when the library is missing or was built against another ABI,
so a GPU run can never silently fall back to something else.
"""
import ctypes
import os
from ctypes import POINTER, c_double, c_int, c_int32, c_int64, c_uint32, c_uint64, c_void_p

MAXN = 16
MAXC = 8
MAXF = 64
NGROUPS = 8
ABI_VERSION = 1

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libimenv.so")

# constants mirrored from include/imenv.h
OK = 0
E_INVALID, E_UNSUPPORTED, E_HIP, E_DONE, E_NOT_RESET, E_SPLIT_LOOP = -1, -2, -3, -4, -5, -6
KIND = {"IM": 0, "MAIM": 1, "IM_div": 2, "MAIM_div": 3}
DECODE_CLIP_ROUND, DECODE_ROUND_CLIP = 0, 1
REWARD_SUM, REWARD_SHARED_MEAN, REWARD_INDEPENDENT = 0, 1, 2
G_INV, G_BACKLOG, G_ORDER_U, G_DEMAND_HIST, G_ORDER_HIST, G_TRANSIT, G_NODE_ID, G_ZERO = range(8)
OBS_ZERO, OBS_RAW, OBS_SCALED, OBS_CLAMP_SCALED = 0, 1, 2, 3
DEMAND_CUSTOM, DEMAND_POISSON, DEMAND_UNIFORM = 1, 2, 3
LAYOUT_DRAW, LAYOUT_PER_ENV, LAYOUT_BROADCAST = 0, 1, 2
F32, F64 = 0, 1
STORE_DEFAULT, STORE_STREAM, STORE_PLAIN, STORE_WRITETHROUGH = 0, 1, 2, 3
PLAN_SHARED, PLAN_PER_EPISODE = 0, 1
STAT_RETURN, STAT_OBJECTIVE, STAT_INVENTORY, STAT_BACKLOG, STAT_CUSTOMER_BACKLOG = range(5)
NUM_STATS = 5
STAT_NAMES = ("return", "objective", "inventory", "backlog", "customer_backlog")
METRIC_NAMES = ("episode_reward", "total_inventory", "total_backlog", "customer_backlog")   # + stage_reward[N]


class ImEnvNativeError(RuntimeError):
    pass


class ImEnvSpec(ctypes.Structure):
    _fields_ = [
        ("abi_version", c_int32), ("kind", c_int32), ("num_nodes", c_int32), ("num_periods", c_int32),
        ("parent", c_int32 * MAXN), ("num_children", c_int32 * MAXN), ("children", (c_int32 * MAXC) * MAXN),
        ("demand_parent", c_int32 * MAXN), ("retailer_slot", c_int32 * MAXN), ("num_retailers", c_int32),
        ("delay", c_int32 * MAXN), ("init_inv", c_int32 * MAXN), ("inv_max", c_int32 * MAXN),
        ("order_max", c_int32 * MAXN), ("backlog_cap", c_int32 * MAXN), ("split_limit", (c_int32 * 4) * MAXN),
        ("sell_price", c_double * MAXN), ("buy_price", c_double * MAXN), ("stock_cost", c_double * MAXN),
        ("backlog_cost", c_double * MAXN), ("inv_target", c_double * MAXN),
        ("standardise_actions", c_int32), ("decode_mode", c_int32), ("a", c_double), ("b", c_double),
        ("reward_mode", c_int32),
        ("num_features", c_int32), ("feat_group", c_int32 * MAXF), ("feat_index", c_int32 * MAXF),
        ("group_mode", c_int32 * NGROUPS), ("group_den", (c_double * MAXN) * NGROUPS),
        ("group_clip", (c_double * MAXN) * NGROUPS), ("prev_length", c_int32),
        ("demand_dist", c_int32), ("poisson_mu", c_double), ("uniform_low", c_int32), ("uniform_high", c_int32),
        ("noisy_demand", c_int32), ("noisy_demand_threshold", c_double),
        ("noisy_delay", c_int32), ("noisy_delay_threshold", c_double),
        ("seed", c_uint64),
    ]


class ImEnvInfo(ctypes.Structure):
    _fields_ = [("order", c_void_p), ("demand", c_void_p), ("acquisition", c_void_p), ("ship", c_void_p),
                ("profit", c_void_p), ("ship_to", c_void_p), ("backlog_to", c_void_p)]


class ImEnvRollout(ctypes.Structure):
    _fields_ = [("policy", c_void_p), ("num_policies", c_int64), ("num_scenarios", c_int64),
                ("demand", c_void_p), ("scenario_offset", c_int64), ("episode", c_int64),
                ("demand_pmf", c_void_p), ("pmf_len", c_int32), ("noisy_delay", c_int32),
                ("noisy_delay_threshold", c_double), ("episode_stats", c_void_p), ("policy_stats", c_void_p)]


class ImEnvPlanRollout(ctypes.Structure):
    _fields_ = [("actions", c_void_p), ("action_dtype", c_int32), ("plan_layout", c_int32),
                ("num_plans", c_int64), ("num_scenarios", c_int64), ("demand", c_void_p),
                ("scenario_offset", c_int64), ("episode", c_int64), ("noisy_delay", c_int32), ("pad_", c_int32),
                ("noisy_delay_threshold", c_double), ("rewards", c_void_p), ("episode_stats", c_void_p),
                ("policy_stats", c_void_p)]


# (name, restype, argtypes) for every symbol include/imenv.h declares
SYMBOLS = [
    ("imenv_create", c_int, [POINTER(ImEnvSpec), c_int64, c_int64, c_int, POINTER(c_void_p)]),
    ("imenv_reset", c_int, [c_void_p, c_void_p, c_int, c_int, c_double, c_void_p, c_int64, c_void_p, c_int,
                            c_void_p]),
    ("imenv_step", c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, POINTER(ImEnvInfo),
                           POINTER(c_int32), c_void_p]),
    ("imenv_base_stock_rollout", c_int, [c_void_p, POINTER(ImEnvRollout), c_void_p]),
    ("imenv_plan_rollout", c_int, [c_void_p, POINTER(ImEnvPlanRollout), c_void_p]),
    ("imenv_set_episode_metrics", c_int, [c_void_p, c_void_p]),
    ("imenv_column_stats", c_int, [c_void_p, c_int64, c_int32, c_void_p, c_void_p]),
    ("imenv_cc_observation", c_int, [c_int64, c_int32, c_int32, c_void_p, c_int, c_void_p, c_int, c_double, c_double,
                                     c_void_p, c_void_p]),
    ("imenv_gae", c_int, [c_int64, c_int32, c_void_p, c_int, c_void_p, c_int, c_void_p, c_double, c_double, c_void_p,
                          c_void_p, c_void_p]),
    ("imenv_get_state", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, POINTER(c_int32), c_void_p]),
    ("imenv_get_errors", c_int, [c_void_p, c_void_p, POINTER(c_uint32), c_void_p]),
    ("imenv_dims", c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]),
    ("imenv_poisson_table", c_int, [c_void_p, POINTER(c_uint32), c_int32, POINTER(c_int32)]),
    ("imenv_state_layout", c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]),
    ("imenv_split_layout", c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32)]),
    ("imenv_draw_layout", c_int, [c_void_p, POINTER(c_int32)]),
    ("imenv_set_delay_uniforms", c_int, [c_void_p, c_int32, c_void_p, c_void_p]),
    ("imenv_set_jit", c_int, [c_void_p, c_int]),
    ("imenv_set_store_policy", c_int, [c_void_p, c_int]),
    ("imenv_debug_stamps", c_int, [c_void_p, c_void_p, c_int64, POINTER(c_int64)]),
    ("imenv_kernel_info", c_int, [c_void_p, ctypes.c_char_p, c_int64]),
    ("imenv_jit_check", c_int, [POINTER(ImEnvSpec), ctypes.c_char_p, c_uint32, ctypes.c_char_p, c_int64]),
    ("imenv_destroy", None, [c_void_p]),
    ("imenv_last_error", ctypes.c_char_p, []),
    ("imenv_abi_version", c_int, []),
    ("imenv_spec_size", c_int64, []),
]

_lib = None


def load(path=None):
    """Load libimenv.so (once). Raises ImEnvNativeError if absent or mismatched."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImEnvNativeError(
            "libimenv.so not found at %s — build it with `python __graft_entry__.py build` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback" % p)
    lib = ctypes.CDLL(p)
    for name, res, args in SYMBOLS:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.imenv_abi_version() != ABI_VERSION:
        raise ImEnvNativeError("libimenv ABI %d != binding ABI %d" % (lib.imenv_abi_version(), ABI_VERSION))
    if lib.imenv_spec_size() != ctypes.sizeof(ImEnvSpec):
        raise ImEnvNativeError("ImEnvSpec layout mismatch: library %d bytes, binding %d bytes"
                               % (lib.imenv_spec_size(), ctypes.sizeof(ImEnvSpec)))
    if path is None:
        _lib = lib
    return lib


def check(rc, what):
    if rc != OK:
        msg = load().imenv_last_error().decode(errors="replace")
        raise ImEnvNativeError("%s failed (%d): %s" % (what, rc, msg))

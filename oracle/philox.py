"""Philox4x32-10 counter RNG and the demand samplers built on it — NumPy restatement.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). The product draws the same
numbers inside the HIP step kernel (marl-for-im_amd/csrc/imenv_device.h,
``rng_word`` / ``rng_block`` in ``step_body`` and ``rollout_body``); this module lets the tests check those
in-kernel draws bit-exactly on the CPU.

Why this exists: the reference draws the whole demand horizon at ``reset()`` from
SciPy's ``poisson.rvs`` / ``randint.rvs`` on NumPy's global legacy MT19937 stream
(environments/IM_env.py:184-207, IM_div_env.py:221-255). That stream is not
reproduced on the GPU; the parity path feeds host-drawn demand instead (as the
reference's own evaluation harness does, inv_management.py:569). The throughput
path draws demand with a counter-based generator keyed by (seed, global env id),
so every env's stream is independent of how envs are sharded over GPUs.

Algorithm (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3", SC'11;
Random123 ``philox4x32_R(10, ...)``), pinned by the published known-answer vectors
in tests/test_oracle_golden.py (KAT tests).

Counter layout used by the product (all uint32):
    c0 = global env id, c1 = episode, c2 = period t // 4, c3 = (stream << 16) | lane
and the word for period t is output word t % 4, so one Philox block serves four consecutive
periods (lane = retailer row, for demand and noisy-demand draws). Noisy delay (one word per node
per period) uses c2 = t, c3 = (stream << 16) | node // 4 and output word node % 4: one block
serves four nodes of one period (``node_word``).
Key: (seed & 0xffffffff, seed >> 32).
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

# Stream ids (counter word c3 high half); must match imenv_device.h.
STREAM_DEMAND = 0
STREAM_NOISY_DEMAND_DOUBLE = 1
STREAM_NOISY_DEMAND_ZERO = 2
STREAM_NOISY_DELAY = 3


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10. Inputs broadcastable uint32 arrays; returns 4 uint32 arrays."""
    c0 = np.asarray(c0, dtype=np.uint32).astype(np.uint64)
    c1 = np.asarray(c1, dtype=np.uint32).astype(np.uint64)
    c2 = np.asarray(c2, dtype=np.uint32).astype(np.uint64)
    c3 = np.asarray(c3, dtype=np.uint32).astype(np.uint64)
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    for r in range(10):
        if r > 0:
            k0 = np.uint32((int(k0) + int(W0)) & 0xFFFFFFFF)
            k1 = np.uint32((int(k1) + int(W1)) & 0xFFFFFFFF)
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        n0 = hi1 ^ c1 ^ np.uint64(k0)
        n1 = lo1
        n2 = hi0 ^ c3 ^ np.uint64(k1)
        n3 = lo0
        c0, c1, c2, c3 = n0, n1, n2, n3
    return (c0.astype(np.uint32), c1.astype(np.uint32),
            c2.astype(np.uint32), c3.astype(np.uint32))


def stream_word(gid, ep, t, stream, lane, k0, k1):
    """The product's random word for (stream, lane, period t): word t % 4 of the Philox block with
    counter (gid, ep, t // 4, stream << 16 | lane) (imenv_device.h rng_word)."""
    return philox4x32_10(gid, ep, int(t) >> 2, (int(stream) << 16) | int(lane), k0, k1)[int(t) & 3]


def node_word(gid, ep, t, stream, node, k0, k1):
    """Noisy-delay word for (node, period t): word node % 4 of the Philox block with counter
    (gid, ep, t, stream << 16 | node // 4) (imenv_device.h rng_node_block)."""
    return philox4x32_10(gid, ep, int(t), (int(stream) << 16) | (int(node) >> 2), k0, k1)[int(node) & 3]


def split_seed(seed):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return seed & 0xFFFFFFFF, seed >> 32


def poisson_thresholds(mu):
    """Integer CDF thresholds for inversion sampling of Poisson(mu) from one uint32.

    thr[k] = ceil(CDF(k) * 2^32) for k = 0..K-2; the sample is the smallest k with
    x < thr[k], or K-1 when no threshold exceeds x (the table is extended until
    the remaining tail is < 2^-32). CDF by the pmf recurrence p_k = p_{k-1} mu / k
    in float64 (same formula, same IEEE ops as the host spec builder).
    """
    mu = float(mu)
    if not (mu > 0.0):
        raise ValueError("Poisson mean must be positive")
    p = np.exp(-mu)
    cdf = 0.0
    thr = []
    k = 0
    while True:
        cdf += p
        t = int(np.ceil(cdf * 4294967296.0))
        if t >= 4294967296 or k >= 4095:
            break
        thr.append(t)
        k += 1
        p = p * mu / k
    return np.array(thr, dtype=np.uint64)


def sample_from_thresholds(x, thr):
    """Smallest k with x < thr[k]; len(thr) if none (vectorised over x)."""
    x = np.asarray(x, dtype=np.uint64)
    return np.searchsorted(thr, x, side="right").astype(np.int64)


def uniform_int(x, low, high):
    """low + floor(x * (high - low) / 2^32): randint[low, high) from one uint32."""
    rng = np.uint64(int(high) - int(low))
    return (int(low) + ((np.asarray(x, dtype=np.uint64) * rng) >> np.uint64(32)).astype(np.int64))


def prob_threshold(p):
    """uint32 threshold T so that (x < T) has probability p (quantised to 2^-32)."""
    t = int(np.ceil(float(p) * 4294967296.0))
    return min(max(t, 0), 4294967296)

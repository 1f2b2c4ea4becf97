"""gym.spaces.Box when gym is importable, else a minimal stand-in with the same fields.

The reference builds its spaces with gym.spaces.Box (environments/IM_env.py:60-160); RLlib reads
only .shape, .dtype, .low, .high and calls .sample() / .contains(). gym is not installed in this
image, so the stand-in keeps the adaptors usable without it.
"""
import numpy as np

try:  # pragma: no cover - exercised only where gym is installed
    from gym.spaces import Box  # noqa: F401
except Exception:  # gym absent (this image)
    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            if shape is None:
                shape = np.shape(low) if np.ndim(low) else np.shape(high)
            self.shape = tuple(int(s) for s in shape)
            self.low = np.broadcast_to(np.asarray(low, dtype=np.float64), self.shape).astype(self.dtype)
            self.high = np.broadcast_to(np.asarray(high, dtype=np.float64), self.shape).astype(self.dtype)
            self._rng = np.random.default_rng()

        def sample(self):
            lo = np.where(np.isfinite(self.low), self.low, -1e6).astype(np.float64)
            hi = np.where(np.isfinite(self.high), self.high, 1e6).astype(np.float64)
            if np.issubdtype(self.dtype, np.integer):
                return self._rng.integers(lo, hi + 1).astype(self.dtype)
            return self._rng.uniform(lo, hi).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

        def __contains__(self, x):
            return self.contains(x)

        def __repr__(self):
            return "Box(%s, %s)" % (self.shape, self.dtype)

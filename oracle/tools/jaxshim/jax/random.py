"""jax.random.PRNGKey / normal via the legacy threefry2x32 generator.

TEST INFRASTRUCTURE ONLY.  Restates JAX's published (pre-0.5 default,
non-partitionable) algorithm: counts = iota(size) split in two halves
(padded to even), threefry2x32 with 20 rounds, bits -> float in [1,2) via
(b >> 9) | 0x3F800000, minus 1, affine map onto [nextafter(-1, 0), 1), then
sqrt(2) * erfinv.  The reference draws J = I + jgm * normal(PRNGKey(0), (3,3))
(trajectory.py:42).
"""
import numpy as _np
from scipy.special import erfinv as _erfinv

from .numpy import _canon

_ROT = ((13, 15, 26, 6), (17, 29, 16, 24))


def PRNGKey(seed):
    seed = int(seed)
    return _np.array([(seed >> 32) & 0xFFFFFFFF, seed & 0xFFFFFFFF], dtype=_np.uint32)


def _rotl(v, r):
    return ((v << _np.uint32(r)) | (v >> _np.uint32(32 - r))).astype(_np.uint32)


def threefry2x32(key, x0, x1):
    with _np.errstate(over="ignore"):
        k0, k1 = _np.uint32(key[0]), _np.uint32(key[1])
        ks = (k0, k1, _np.uint32(k0 ^ k1 ^ _np.uint32(0x1BD11BDA)))
        x = [(x0 + ks[0]).astype(_np.uint32), (x1 + ks[1]).astype(_np.uint32)]

        def rounds(x, rots):
            for r in rots:
                x[0] = (x[0] + x[1]).astype(_np.uint32)
                x[1] = _rotl(x[1], r)
                x[1] = (x[0] ^ x[1]).astype(_np.uint32)
            return x

        inj = [(1, 2), (2, 0), (0, 1), (1, 2), (2, 0)]
        for i in range(5):
            x = rounds(x, _ROT[i % 2])
            a, b = inj[i]
            x[0] = (x[0] + ks[a]).astype(_np.uint32)
            x[1] = (x[1] + ks[b] + _np.uint32(i + 1)).astype(_np.uint32)
        return x[0], x[1]


def random_bits(key, shape):
    size = int(_np.prod(shape))
    counts = _np.arange(size, dtype=_np.uint32)
    odd = size % 2
    if odd:
        counts = _np.concatenate([counts, _np.zeros(1, dtype=_np.uint32)])
    half = counts.size // 2
    y0, y1 = threefry2x32(key, counts[:half], counts[half:])
    out = _np.concatenate([y0, y1])
    if odd:
        out = out[:-1]
    return out.reshape(shape)


def uniform(key, shape, minval, maxval):
    bits = random_bits(key, shape)
    fbits = (bits >> _np.uint32(9)) | _np.uint32(0x3F800000)
    floats = fbits.view(_np.float32) - _np.float32(1.0)
    minval, maxval = _np.float32(minval), _np.float32(maxval)
    return _np.maximum(minval, floats * (maxval - minval) + minval).astype(_np.float32)


def normal(key, shape=(), dtype=None):
    lo = _np.nextafter(_np.float32(-1.0), _np.float32(0.0), dtype=_np.float32)
    u = uniform(key, tuple(shape), lo, 1.0)
    z = _np.float32(_np.sqrt(2.0)) * _erfinv(u.astype(_np.float64)).astype(_np.float32)
    return _canon(z.astype(_np.float32))

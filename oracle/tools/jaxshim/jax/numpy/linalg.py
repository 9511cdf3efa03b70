"""jax.numpy.linalg subset on numpy/LAPACK (test infrastructure only)."""
import numpy as _np

from . import _canon, _plain, _promote


def solve(a, b):
    a, b = _promote([_plain(a), _plain(b)])
    return _canon(_np.linalg.solve(a, b))


def inv(a):
    return _canon(_np.linalg.inv(_plain(a)))


def norm(x, ord=None, axis=None):
    return _canon(_np.linalg.norm(_plain(x), ord=ord, axis=axis))

"""numpy-backed stand-in for the subset of `jax.numpy` the reference uses.

TEST INFRASTRUCTURE ONLY (see ../__init__.py).  Mirrors JAX's default
(x64-disabled) type rules: every floating result is float32, every integer
result int32, int32 arrays combined with floats promote to float32 (not
float64 as plain numpy would), and arrays support `.at[idx].set(v)`.
Set IRM_JAXSHIM_X64=1 to compute in float64 instead (finite-difference checks).
Set IRM_JAXSHIM_MATMUL=exact to accumulate every `@` (matmul) in float64 and round the result
once to float32 — the correctly rounded contraction the build's kernels and C oracle use — while
every other operation keeps the reference's fp32 arithmetic (gen_golden_bench.py's "_xm" fixtures).
"""
import os

import numpy as _np

_X64 = os.environ.get("IRM_JAXSHIM_X64", "0") == "1"
_XMATMUL = os.environ.get("IRM_JAXSHIM_MATMUL", "") == "exact"
FLOAT = _np.float64 if _X64 else _np.float32
INT = _np.int64 if _X64 else _np.int32

newaxis = None
float32 = _np.float32
int32 = _np.int32
uint32 = _np.uint32


def _canon(x):
    """Cast a numpy result to JAX's default dtypes and wrap arrays."""
    if isinstance(x, tuple):
        return tuple(_canon(v) for v in x)
    if isinstance(x, list):
        return [_canon(v) for v in x]
    if isinstance(x, _np.ndarray):
        if x.dtype.kind == "f" and x.dtype != FLOAT:
            x = x.astype(FLOAT)
        elif x.dtype.kind in "iu" and x.dtype.itemsize == 8 and not _X64 and x.dtype != _np.uint64:
            x = x.astype(_np.int32 if x.dtype.kind == "i" else _np.uint32)
        return x.view(JArray)
    if isinstance(x, _np.generic):
        if x.dtype.kind == "f" and x.dtype != FLOAT:
            return FLOAT(x)
        if x.dtype.kind == "i" and x.dtype.itemsize == 8 and not _X64:
            return _np.int32(x)
        return x
    if isinstance(x, float):
        return x
    return x


def _plain(x):
    if isinstance(x, JArray):
        return x.view(_np.ndarray)
    return x


def _promote(args):
    """JAX promotion: any float operand => integer arrays become FLOAT."""
    has_float = any(
        (isinstance(a, (_np.ndarray, _np.generic)) and a.dtype.kind == "f") or isinstance(a, float)
        for a in args
    )
    if not has_float:
        return args
    out = []
    for a in args:
        if isinstance(a, (_np.ndarray, _np.generic)) and a.dtype.kind in "iu":
            a = a.astype(FLOAT)
        out.append(a)
    return out


class _AtSetter:
    def __init__(self, arr, idx):
        self._arr, self._idx = arr, idx

    def set(self, value):
        out = _np.array(self._arr.view(_np.ndarray), copy=True)
        out[self._idx] = _plain(value)
        return _canon(out)


class _AtIndexer:
    def __init__(self, arr):
        self._arr = arr

    def __getitem__(self, idx):
        return _AtSetter(self._arr, idx)


class JArray(_np.ndarray):
    """ndarray with JAX dtype rules and the functional `.at[]` update."""

    def __array_ufunc__(self, ufunc, method, *inputs, **kwargs):
        args = [_plain(a) for a in inputs]
        if _XMATMUL and ufunc is _np.matmul and method == "__call__":
            args = [a.astype(_np.float64) if isinstance(a, _np.ndarray) else a for a in _promote(args)]
            return _canon(_np.matmul(*args).astype(FLOAT))
        if ufunc not in (_np.logical_and, _np.logical_or, _np.logical_not, _np.invert):
            args = _promote(args)
        kwargs.pop("out", None)
        res = getattr(ufunc, method)(*args, **kwargs)
        return _canon(res)

    @property
    def at(self):
        return _AtIndexer(self)


def _wrap(fn):
    def inner(*args, **kwargs):
        args = [_plain(a) for a in args]
        kwargs = {k: _plain(v) for k, v in kwargs.items()}
        return _canon(fn(*args, **kwargs))

    inner.__name__ = getattr(fn, "__name__", "fn")
    return inner


def _wrap_promote(fn):
    def inner(*args, **kwargs):
        args = _promote([_plain(a) for a in args])
        kwargs = {k: _plain(v) for k, v in kwargs.items()}
        return _canon(fn(*args, **kwargs))

    inner.__name__ = getattr(fn, "__name__", "fn")
    return inner


def array(obj, dtype=None):
    a = _np.array(_plain(obj) if not isinstance(obj, (list, tuple)) else [_plain(o) for o in obj], dtype=dtype)
    return _canon(a)


asarray = array


def linspace(start, stop, num, dtype=None):
    """fp32 linspace as jnp computes it: t_i = start*(1-i/div) + stop*(i/div)."""
    num = int(num)
    if num == 1:
        return _canon(_np.array([start], dtype=FLOAT))
    div = FLOAT(num - 1)
    step = _np.arange(num - 1, dtype=FLOAT) / div
    out = FLOAT(start) * (FLOAT(1) - step) + FLOAT(stop) * step
    out = _np.concatenate([out, _np.array([stop], dtype=FLOAT)])
    return _canon(out.astype(FLOAT))


def eye(n, m=None, dtype=None):
    return _canon(_np.eye(n, m, dtype=dtype or FLOAT))


def ones(shape, dtype=None):
    return _canon(_np.ones(shape, dtype=dtype or FLOAT))


def zeros(shape, dtype=None):
    return _canon(_np.zeros(shape, dtype=dtype or FLOAT))


def zeros_like(a, dtype=None):
    return _canon(_np.zeros_like(_plain(a), dtype=dtype))


exp = _wrap(_np.exp)
cos = _wrap(_np.cos)
sin = _wrap(_np.sin)
sqrt = _wrap(_np.sqrt)
abs = _wrap(_np.abs)  # noqa: A001
square = _wrap(_np.square)
cumsum = _wrap(_np.cumsum)
max = _wrap(_np.max)  # noqa: A001
min = _wrap(_np.min)  # noqa: A001
sum = _wrap(_np.sum)  # noqa: A001
argmax = _wrap(_np.argmax)
meshgrid = _wrap(_np.meshgrid)
expand_dims = _wrap(_np.expand_dims)
logical_and = _wrap(_np.logical_and)
logical_or = _wrap(_np.logical_or)
multiply = _wrap_promote(_np.multiply)
einsum = _wrap_promote(_np.einsum)
where = _wrap_promote(_np.where)


def stack(arrays, axis=0):
    return _canon(_np.stack(_promote([_plain(a) for a in arrays]), axis=axis))


def concatenate(arrays, axis=0):
    return _canon(_np.concatenate(_promote([_plain(a) for a in arrays]), axis=axis))


from . import linalg  # noqa: E402,F401

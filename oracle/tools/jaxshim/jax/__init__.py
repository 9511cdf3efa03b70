"""Minimal numpy adapter exposing the slice of the public `jax` API that the
reference (simongroeger/irm_motion_planning) uses.

TEST INFRASTRUCTURE ONLY.  `jax`/`jaxlib` are not installed in the build
container and there is no network, so this adapter lets the *unmodified*
reference sources under /root/reference import and run, purely to generate
golden vectors (tests/golden/) and to pin oracle/ against them.  It never
ships to the GPU box's product path and nothing in irm_motion_planning_amd/
imports it.

Semantics mirrored from JAX's documented behaviour:
  * default dtype float32 / int32 (jax_enable_x64 off),
  * `jit` / `lax.while_loop` / `lax.cond` are the eager Python equivalents,
  * `random.PRNGKey` / `random.normal` follow the legacy (non-partitionable)
    threefry2x32 generator, see random.py.
"""
import contextlib
import functools

from . import numpy  # noqa: F401
from . import lax  # noqa: F401
from . import random  # noqa: F401
from . import profiler  # noqa: F401


class _Config:
    def update(self, *args, **kwargs):
        return None


config = _Config()


def jit(fun=None, **kwargs):
    """Identity: eager execution has jit's semantics for this code base."""
    if fun is None:
        return functools.partial(jit, **kwargs)
    return fun


def block_until_ready(x):
    return x


@contextlib.contextmanager
def _null_ctx(*a, **k):
    yield


Array = numpy.JArray

"""No-op stand-in for jax.profiler (test infrastructure only)."""
import contextlib


@contextlib.contextmanager
def trace(*args, **kwargs):
    yield

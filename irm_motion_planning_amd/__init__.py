"""MI355X-native (gfx950 / CDNA4) RKHS trajectory optimiser.

Drop-in for the hot path of simongroeger/irm_motion_planning: the functional
gradient-descent / backtracking-line-search inner loop (optimizer_GD.py,
optimizer_BLS.py) over trajectory.py / robot.py / environment.py.  The Python
classes here mirror the reference's object API; all numerics run in the
hand-written HIP kernels of csrc/ behind the C ABI of include/irm.h.
"""
from ._abi import IrmError, load_library  # noqa: F401

__all__ = ["IrmError", "load_library"]

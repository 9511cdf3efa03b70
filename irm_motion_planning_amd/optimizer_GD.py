"""GradientDescentOptimizer — mirrors optimizer_GD.py (optimizer_GD.py:14-232).

Fixed-step functional gradient descent.  With max_outer_iteration > 1 it is
the dual loop (jit_dual_optimize, optimizer_GD.py:173-232: per-outer step
size gd_lr[outer], λ escalation on violated constraints); with 1 it is the
single loop (jit_optimize, optimizer_GD.py:68-97).  Both run on device in
one persistent launch: k_lean for the specialised shapes (the bench path),
k_optimize otherwise (the library's launch plan names the kernel).
"""
from ._abi import IrmError
from ._optimizer import _PersistentOptimizer


class GradientDescentOptimizer(_PersistentOptimizer):
    kind = "gd"

    def __init__(self, args, **overrides):
        self.dualOptimization = args.max_outer_iteration > 1
        if args.max_outer_iteration > len(args.gd_lr):  # optimizer_GD.py:34-36
            print("FATAL: max_outer_iteration and dual_lr do not match")
            raise IrmError("max_outer_iteration and dual_lr do not match")
        self.dual_lr = list(args.gd_lr)
        self.lr = self.dual_lr[0]
        super().__init__(args, **overrides)

    def optimize(self):
        out = super().optimize()
        if not self.jitLoop and not self.dualOptimization and self.last_stats is not None:
            # plain_optimize prints where the single loop stopped (optimizer_GD.py:111)
            if int(self.last_stats["inner_iterations"]) < self.max_inner_iteration:
                print("break after", int(self.last_stats["inner_iterations"]), "iteration")
        return out

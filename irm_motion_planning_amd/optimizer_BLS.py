"""BacktrackingLineSearchOptimizer — mirrors optimizer_BLS.py (optimizer_BLS.py:22-213).

Squared-penalty dual loop with normalised-gradient steps and Armijo
backtracking (trial loop optimizer_BLS.py:131-150, inner loop 154-179, outer
loop 183-211), all inside one persistent launch (k_lean for the specialised
shapes: the search direction is computed once per inner iteration and every
trial step is a per-waypoint evaluation; k_optimize otherwise: each trial's
fp32 iterate evaluated exactly).
"""
from ._optimizer import _PersistentOptimizer


class BacktrackingLineSearchOptimizer(_PersistentOptimizer):
    kind = "bls"

    def __init__(self, args, **overrides):
        self.bls_max_iter = args.max_bls_iteration
        self.bls_lr_start = args.bls_lr_start
        self.bls_alpha = args.bls_alpha
        self.bls_beta_minus = args.bls_beta_minus
        self.bls_beta_plus = args.bls_beta_plus
        super().__init__(args, **overrides)

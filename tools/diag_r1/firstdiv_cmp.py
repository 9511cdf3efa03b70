import sys
import numpy as np
a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for k in (1, 2, 3, 5, 10, 15):
    for name in ("alpha", "traj", "loss"):
        x0, x1, y0 = a[f"k{k}_r0_{name}"], a[f"k{k}_r1_{name}"], b[f"k{k}_r0_{name}"]
        y1 = b[f"k{k}_r1_{name}"]
        d = np.abs(x0.astype(np.float64) - y0).max()
        nd = int(np.sum(x0 != y0))
        print(f"k={k:2d} {name:5s} def-rep {np.array_equal(x0, x1)} ilp-rep {np.array_equal(y0, y1)}  def vs ilp: {nd} elements differ, max {d:.3e}")

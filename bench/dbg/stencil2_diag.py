"""Where the two-step stencil walk differs from two one-step launches (diagnostics)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from cme213_sp18_amd.suite import hw3
for (nx, ny, it) in [(9, 9, 2), (64, 64, 2), (257, 131, 2), (300, 64, 2), (64, 300, 2)]:
    p = hw3.SimParams(nx, ny, 1.0, 1.0, it, 8)
    g0 = hw3.init_grid(p)
    a, _ = hw3.gpu_computation(g0, p, "shared")
    b, _ = hw3.gpu_computation(g0, p, "shared2")
    ref = hw3.cpu_computation(g0, p)
    d = np.argwhere(a != b)
    rows = sorted(set(d[:, 0].tolist())); cols = sorted(set(d[:, 1].tolist()))
    u = hw3.ulp_distance(a, b)
    print(nx, ny, it, "diff", len(d), "rows", rows[:12], len(rows), "cols", cols[:16], len(cols), "max ulp", int(u.max()),
          "| vs cpu: shared", int(hw3.ulp_distance(ref, a).max()), "shared2", int(hw3.ulp_distance(ref, b).max()), flush=True)

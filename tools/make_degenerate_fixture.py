#!/usr/bin/env python3
"""tests/golden/degenerate_inliers.npz: the refit inlier sets of the bench regimes whose design
matrix has a null space of dimension > 1 (the sets where the refit's power iteration reaches its
32-step cap).  Found by running the oracle's trajectory loop (tests/test_svd_tolerance.py's
restatement) over 200-frame scene sequences at 1.0 and 0.12 m/frame.  Fixture data for
test_oracle_kat.py / test_gpu_parity.py (the solver's certified exit)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O  # noqa: E402
import test_svd_tolerance as T  # noqa: E402

out = {}
for step in (1.0, 0.12):
    recs = T._run_sequence(step)[0]
    for r in recs:
        if r["status"] != 0:
            out[f"step{step}_frame{r['frame']}"] = r["P"]
            print(step, r["frame"], r["P"].shape[0], "status", r["status"])
np.savez_compressed(os.path.join(ROOT, "tests", "golden", "degenerate_inliers.npz"), **out)

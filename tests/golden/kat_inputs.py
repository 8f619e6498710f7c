"""Deterministic inputs of the quantile known-answer tests (regenerated, not stored)."""
import numpy as np


def quantile_inputs():
    cases = {}
    rng = np.random.default_rng(123)
    a = rng.standard_normal((10007, 140)).astype(np.float32)
    a[:, 3] = 0.5                      # constant column
    a[::7, 5] = 1.25                   # heavy ties
    a[:, 6] = np.round(a[:, 6] * 4) / 4
    cases["big"] = a
    cases["n1"] = rng.standard_normal((1, 140)).astype(np.float32)
    cases["n2"] = rng.standard_normal((2, 140)).astype(np.float32)
    cases["n101"] = rng.standard_normal((101, 140)).astype(np.float32)
    cases["n3000"] = (rng.standard_normal((3000, 140)) * 1e-3).astype(np.float32)
    return cases

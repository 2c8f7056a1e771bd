"""Synthetic inputs shared by the development tools and bench.py."""
import numpy as np


def euclid(n, seed=1, dim=8):
    """Packed LT (reference order) of Euclidean distances between n random
    points in [0,1)^dim, rounded to 9 decimals like a Phylip matrix."""
    rng = np.random.default_rng(seed)
    pts = rng.random((n, dim))
    D = np.empty(n * (n - 1) // 2)
    for i in range(1, n):
        o = i * (i - 1) // 2
        D[o:o + i] = np.sqrt(((pts[:i] - pts[i]) ** 2).sum(1))
    return np.round(D * 1e9) / 1e9

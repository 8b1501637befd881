"""``core/geometry.py`` surface used on the hot path.

The batched engine computes separating vectors on the GPU (inside the fused kernel); this host
helper keeps the reference's public function for callers that use it directly.
"""
from __future__ import annotations

import numpy as np


def compute_separating_vector(ego_pos, obstacle_pos):
    """Unit vector from ``ego_pos`` to ``obstacle_pos``; ``[1, 0]`` when they are closer than
    1e-10 (``core/geometry.py:35-53``)."""
    diff = np.asarray(obstacle_pos, dtype=np.float64) - np.asarray(ego_pos, dtype=np.float64)
    norm = np.linalg.norm(diff)
    if norm < 1e-10:
        return np.array([1.0, 0.0])
    return diff / norm

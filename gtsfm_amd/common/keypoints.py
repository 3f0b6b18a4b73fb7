"""Keypoints container with the reference's API (gtsfm/common/keypoints.py:15-231).

Coordinates are (x, y) with x to the right, y down, origin at the top-left pixel corner (keypoints.py:18-21).
The reference cannot be imported on the GPU box, so the product re-declares this type; attribute names, dtypes
and `get_top_k` / `extract_indices` semantics follow the reference.
"""
from __future__ import annotations

import copy
from typing import Optional, Tuple

import numpy as np


def _same(a: Optional[np.ndarray], b: Optional[np.ndarray]) -> bool:
    if a is None or b is None:
        return a is None and b is None
    return np.array_equal(a, b)


class Keypoints:
    """Detections of one image: coordinates (N,2), optional scales (N,) and responses (N,)."""

    def __init__(self, coordinates: np.ndarray, scales: Optional[np.ndarray] = None,
                 responses: Optional[np.ndarray] = None):
        self.coordinates = coordinates
        self.scales = scales
        self.responses = responses

    def __len__(self) -> int:
        return self.coordinates.shape[0]

    def __eq__(self, other: object) -> bool:
        if not isinstance(other, Keypoints):
            return False
        return (_same(self.coordinates, other.coordinates) and _same(self.scales, other.scales)
                and _same(self.responses, other.responses))

    def __ne__(self, other: object) -> bool:
        return not self == other

    def get_top_k(self, k: int) -> Tuple["Keypoints", np.ndarray]:
        """Top-k by response (keypoints.py:89-110). Fewer than k available -> a copy of everything, in order.

        The reference selects with np.argpartition, whose order is implementation-defined; the device path
        emits the top-k in a fixed order (descending response, ties by detection order) instead.
        """
        n = len(self)
        if k >= n:
            return copy.deepcopy(self), np.arange(n)
        if self.responses is None:
            idx = np.arange(k, dtype=np.uint32)
        else:
            idx = np.argpartition(-self.responses, k)[:k]
        return self.extract_indices(idx), idx

    def filter_by_mask(self, mask: np.ndarray) -> Tuple["Keypoints", np.ndarray]:
        """Keeps keypoints whose rounded (x, y) falls on a 1 of the (H, W) mask (keypoints.py:112-125)."""
        xy = np.round(self.coordinates).astype(int)
        keep = np.flatnonzero(mask[xy[:, 1], xy[:, 0]] == 1)
        return self.extract_indices(keep), keep

    def get_x_coordinates(self) -> np.ndarray:
        return self.coordinates[:, 0]

    def get_y_coordinates(self) -> np.ndarray:
        return self.coordinates[:, 1]

    def cast_to_float(self) -> "Keypoints":
        f = lambda a: None if a is None else a.astype(np.float32)  # noqa: E731
        return Keypoints(f(self.coordinates), f(self.scales), f(self.responses))

    def extract_indices(self, indices: np.ndarray) -> "Keypoints":
        if indices.size == 0:
            return Keypoints(coordinates=np.zeros((0, 2)))
        pick = lambda a: None if a is None else a[indices]  # noqa: E731
        return Keypoints(self.coordinates[indices], pick(self.scales), pick(self.responses))

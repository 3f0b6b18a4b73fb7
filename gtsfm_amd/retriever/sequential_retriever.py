"""Sliding-window and exhaustive pair proposals (gtsfm/retriever/sequential_retriever.py:18-58,
exhaustive_retriever.py:12-19). Pure index arithmetic on the host: nothing here touches the device."""
from __future__ import annotations

from pathlib import Path
from typing import List, Optional, Tuple

import numpy as np

from gtsfm_amd.retriever.retriever_base import ImageMatchingRegime, RetrieverBase

MAX_POSSIBLE_FRAME_LOOKAHEAD = 10000  # exhaustive_retriever.py:12


def sequential_pairs(num_images: int, max_frame_lookahead: int) -> np.ndarray:
    """(P, 2) int64 pairs (i1, i2), i1 < i2 <= i1 + max_frame_lookahead, in the reference's loop order (:52-55)."""
    i1, i2 = np.triu_indices(num_images, k=1)
    keep = (i2 - i1) <= max_frame_lookahead
    return np.stack([i1[keep], i2[keep]], axis=1).astype(np.int64)


class SequentialRetriever(RetrieverBase):
    def __init__(self, max_frame_lookahead: int) -> None:
        super().__init__(matching_regime=ImageMatchingRegime.SEQUENTIAL)
        self._max_frame_lookahead = max_frame_lookahead

    def __repr__(self) -> str:
        return f"SequentialRetriever(max_frame_lookahead={self._max_frame_lookahead})"

    def get_image_pairs(self, global_descriptors: Optional[List[np.ndarray]], image_fnames: List[str],
                        plots_output_dir: Optional[Path] = None) -> List[Tuple[int, int]]:
        return [(int(a), int(b)) for a, b in sequential_pairs(len(image_fnames), self._max_frame_lookahead)]


class ExhaustiveRetriever(SequentialRetriever):
    """Every pair (N choose 2): what AllPairsFrontEnd does when given no pair list."""

    def __init__(self) -> None:
        super().__init__(max_frame_lookahead=MAX_POSSIBLE_FRAME_LOOKAHEAD)
        self._matching_regime = ImageMatchingRegime.EXHAUSTIVE

"""Base class of the image-pair retrievers (mirrors gtsfm/retriever/retriever_base.py:17-83).

A retriever proposes the (i1, i2) image pairs the two-view front-end matches and verifies; its output feeds
`AllPairsFrontEnd(image_pairs=...)` (the role of image_pairs_generator.py:29-47). The reference's UI metadata
(GTSFMProcess.get_ui_metadata) is a process-graph drawing aid and is not mirrored.
"""
from __future__ import annotations

import abc
from enum import Enum
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np


class ImageMatchingRegime(str, Enum):
    """retriever_base.py:17-23."""

    SEQUENTIAL: str = "sequential"
    RETRIEVAL: str = "retrieval"
    EXHAUSTIVE: str = "exhaustive"
    SEQUENTIAL_WITH_RETRIEVAL: str = "sequential_with_retrieval"
    RIG_HILTI: str = "rig_hilti"
    SEQUENTIAL_HILTI: str = "sequential_hilti"


class RetrieverBase(abc.ABC):
    """retriever_base.py:26-34."""

    def __init__(self, matching_regime: ImageMatchingRegime) -> None:
        self._matching_regime = matching_regime

    @abc.abstractmethod
    def get_image_pairs(self, global_descriptors: Optional[List[np.ndarray]], image_fnames: List[str],
                        plots_output_dir: Optional[Path] = None) -> List[Tuple[int, int]]:
        """(i1, i2) image pairs to match (retriever_base.py:47-63)."""

    def evaluate(self, num_images: int, image_pair_indices: List[Tuple[int, int]]) -> Dict[str, Dict[str, int]]:
        """The reference's "retriever_metrics" group (retriever_base.py:65-83) as a plain dict."""
        return {"retriever_metrics": {"num_input_images": int(num_images),
                                      "num_retrieved_image_pairs": len(image_pair_indices)}}

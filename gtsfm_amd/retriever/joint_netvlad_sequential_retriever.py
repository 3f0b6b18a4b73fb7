"""Union of NetVLAD and sequential pairs (mirrors gtsfm/retriever/joint_netvlad_sequential_retriever.py:18-80)."""
from __future__ import annotations

from pathlib import Path
from typing import List, Optional, Tuple

from gtsfm_amd.retriever.netvlad_retriever import Descriptors, NetVLADRetriever
from gtsfm_amd.retriever.retriever_base import ImageMatchingRegime, RetrieverBase
from gtsfm_amd.retriever.sequential_retriever import SequentialRetriever


class JointNetVLADSequentialRetriever(RetrieverBase):
    def __init__(self, num_matched: int, min_score: float, max_frame_lookahead: int) -> None:
        super().__init__(matching_regime=ImageMatchingRegime.SEQUENTIAL_WITH_RETRIEVAL)
        self._num_matched = num_matched
        self._similarity_retriever = NetVLADRetriever(num_matched=num_matched, min_score=min_score)
        self._seq_retriever = SequentialRetriever(max_frame_lookahead=max_frame_lookahead)

    def __repr__(self) -> str:
        return f"JointNetVLADSequentialRetriever({self._similarity_retriever}, {self._seq_retriever})"

    def get_image_pairs(self, global_descriptors: Optional[Descriptors], image_fnames: List[str],
                        plots_output_dir: Optional[Path] = None) -> List[Tuple[int, int]]:
        sim_pairs = self._similarity_retriever.get_image_pairs(global_descriptors, image_fnames, plots_output_dir)
        seq_pairs = self._seq_retriever.get_image_pairs(None, image_fnames, plots_output_dir)
        return self._aggregate_pairs(sim_pairs, seq_pairs)

    def _aggregate_pairs(self, sim_pairs: List[Tuple[int, int]],
                         seq_pairs: List[Tuple[int, int]]) -> List[Tuple[int, int]]:
        """The set union (:66-80), sorted (the reference returns it in set-iteration order)."""
        return sorted(set(sim_pairs).union(set(seq_pairs)))

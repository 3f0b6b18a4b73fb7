"""NetVLAD retriever on the MI355X: global-descriptor similarity + top-k image pairs (mirrors
gtsfm/retriever/netvlad_retriever.py:33-228).

The reference computes the similarity matrix as one torch einsum per block pair of the upper block triangle
(`_compute_similarity_subblock`, :109-134), copies the blocks into a zero CPU matrix (:136-149), then masks and
top-k-selects on that matrix (`pairs_from_score_matrix`, :196-228). Here the whole matrix is one fp32-MFMA launch
(gtsfm_retrieval_similarity: 64 x 64 tiles, tiles wholly below the block diagonal skipped and written as zeros) and the
selection one launch with a workgroup per row (gtsfm_retrieval_pairs); only the (i, j) list comes back to the host.
Both kernels live in gtsfm_amd/csrc/retrieval.hip. There is no CPU fallback.

Differences from the reference, all outside the returned pair list unless noted:
- the similarity matrix stays on the device (the reference returns a CPU tensor); `blocksize` only shapes which
  entries are zero, as in the reference, not the launch;
- fp32 accumulation in a different summation order than torch's einsum (|diff| <~ 1e-6 relative): a pair whose
  score ties another to within that rounding may rank differently;
- equal scores rank by ascending column (torch.topk leaves the order of ties unspecified);
- `pairs_from_score_matrix` does not mask its `scores` argument in place (the reference's masked_fill_ does).
The global descriptor network itself (frontend/global_descriptor/netvlad_global_descriptor.py) needs pretrained
weights that are not available offline; descriptors come from the caller.
"""
from __future__ import annotations

import logging
import math
import os
from pathlib import Path
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from gtsfm_amd import device as gdev
from gtsfm_amd import native
from gtsfm_amd.retriever.retriever_base import ImageMatchingRegime, RetrieverBase

logger = logging.getLogger(__name__)
MAX_NUM_IMAGES = 10000  # netvlad_retriever.py:21

Descriptors = Union[Sequence[np.ndarray], np.ndarray, torch.Tensor]


def _dev() -> torch.device:
    native.require_gpu()
    return torch.device("cuda", torch.cuda.current_device())


def _as_device_matrix(global_descriptors: Descriptors) -> torch.Tensor:
    if isinstance(global_descriptors, torch.Tensor):
        d = global_descriptors
    else:
        arr = np.asarray(global_descriptors if len(global_descriptors) else np.zeros((0, 1), np.float32))
        d = torch.from_numpy(np.ascontiguousarray(arr.reshape(arr.shape[0], -1)))
    return d.reshape(d.shape[0], -1).to(device=_dev(), dtype=torch.float32).contiguous()


class NetVLADRetriever(RetrieverBase):
    def __init__(self, num_matched: int, min_score: float = 0.1, blocksize: int = 50) -> None:
        """netvlad_retriever.py:34-44."""
        super().__init__(matching_regime=ImageMatchingRegime.RETRIEVAL)
        self._num_matched = num_matched
        self._blocksize = blocksize
        self._min_score = min_score

    def __repr__(self) -> str:
        return (f"NetVLADRetriever(num_matched={self._num_matched}, blocksize={self._blocksize}, "
                f"min_score={self._min_score})")

    def get_image_pairs(self, global_descriptors: Optional[Descriptors], image_fnames: List[str],
                        plots_output_dir: Optional[Path] = None) -> List[Tuple[int, int]]:
        """netvlad_retriever.py:54-75."""
        if global_descriptors is None:
            raise ValueError("Global descriptors need to be provided")
        sim = self.compute_similarity_matrix(global_descriptors)
        return self.compute_pairs_from_similarity_matrix(sim=sim, image_fnames=image_fnames,
                                                         plots_output_dir=plots_output_dir)

    def compute_similarity_matrix(self, global_descriptors: Descriptors) -> torch.Tensor:
        """(N, N) f32 device tensor: descriptor dot products where j's block >= i's block, 0 elsewhere
        (netvlad_retriever.py:77-149)."""
        num_images = len(global_descriptors)
        if num_images > MAX_NUM_IMAGES:
            raise RuntimeError("Cannot construct similarity matrix of this size.")
        desc = _as_device_matrix(global_descriptors)
        logger.info("NetVLAD similarity: %d images, %d block(s) of %d", num_images,
                    math.ceil(num_images / self._blocksize) if num_images else 0, self._blocksize)
        return gdev.retrieval_similarity(desc, self._blocksize)

    def compute_pairs_from_similarity_matrix(self, sim: torch.Tensor, image_fnames: List[str],
                                             plots_output_dir: Optional[Path] = None) -> List[Tuple[int, int]]:
        """netvlad_retriever.py:151-193: strict upper triangle, min_score, top num_matched per row."""
        num_images = len(image_fnames)
        if tuple(sim.shape) != (num_images, num_images):
            raise AssertionError("scores.shape == invalid.shape")  # the reference's assert (:216)
        sim_d = sim.to(device=_dev(), dtype=torch.float32)
        out, cnt = gdev.retrieval_pairs(sim_d, self._num_matched, self._min_score)
        pairs = _gather_pairs(out, cnt)
        if plots_output_dir:
            _save_plots(sim_d, image_fnames, pairs, Path(plots_output_dir))
        logger.info("Found %d pairs from the NetVLAD Retriever.", len(pairs))
        return pairs


def _gather_pairs(out: torch.Tensor, cnt: torch.Tensor) -> List[Tuple[int, int]]:
    """Rows concatenated in order, each row's first cnt[i] ranks (the reference's np.where(valid) walk, :225-227)."""
    k = out.shape[1]
    if out.shape[0] == 0 or k == 0:
        return []
    keep = torch.arange(k, device=out.device)[None, :] < cnt[:, None]
    sel = out[keep].cpu().numpy()
    return [(int(i), int(j)) for i, j in sel]


def _save_plots(sim: torch.Tensor, image_fnames: List[str], pairs: List[Tuple[int, int]], out_dir: Path) -> None:
    """netvlad_retriever.py:172-190 (matrix image, matrix values, scored named pairs)."""
    os.makedirs(out_dir, exist_ok=True)
    s = sim.detach().cpu().numpy()
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        plt.imshow(np.triu(s))
        plt.title("Image Similarity Matrix")
        plt.savefig(str(out_dir / "netvlad_similarity_matrix.jpg"), dpi=500)
        plt.close("all")
    except ImportError:
        logger.warning("matplotlib unavailable: similarity matrix image not written")
    np.savetxt(fname=str(out_dir / "netvlad_similarity_matrix.txt"), X=s, fmt="%.2f", delimiter=",")
    with open(out_dir / "netvlad_named_pairs.txt", "w") as fid:
        for i, j in pairs:
            fid.write("%.4f %s %s\n" % (s[i, j], image_fnames[i], image_fnames[j]))


def pairs_from_score_matrix(scores: torch.Tensor, invalid: np.ndarray, num_select: int,
                            min_score: Optional[float] = None) -> List[Tuple[int, int]]:
    """netvlad_retriever.py:196-228 on the device: per row, the finite entries of topk(masked scores, num_select)."""
    if tuple(scores.shape) != tuple(np.shape(invalid)):
        raise AssertionError("scores.shape == invalid.shape")
    dev = _dev()
    s = scores.to(device=dev, dtype=torch.float32)
    inv = torch.from_numpy(np.ascontiguousarray(invalid, dtype=bool)).to(dev)
    out, cnt = gdev.retrieval_pairs(s, num_select, min_score, invalid=inv)
    return _gather_pairs(out, cnt)

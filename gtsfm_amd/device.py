"""Device-resident batched entry points over the C ABI (include/gtsfm_hip.h).

torch provides HBM allocations and the stream; every computation is a libgtsfm_hip.so kernel. Tensors passed
in must already live on the GPU; nothing here copies to the host or synchronises.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from gtsfm_amd import native


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _workspace(nbytes: int, device: torch.device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def match_pairs(desc: torch.Tensor, counts: torch.Tensor, pairs: torch.Tensor, ratio: Optional[float],
                mode: int = native.GTSFM_MATCH_INT_F16, stream: Optional[torch.cuda.Stream] = None
                ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Mutual-NN + ratio matching of every (i1, i2) row of `pairs`.

    Args:
        desc: (n_img, kmax, dim) float32 descriptors on the GPU (rows >= counts[i] are ignored).
        counts: (n_img,) int32 valid rows per image.
        pairs: (P, 2) int32 image index pairs.
        ratio: ratio-test threshold, or None for plain mutual NN.
        mode: GTSFM_MATCH_INT_F16 (integer descriptors, MFMA) or GTSFM_MATCH_EXACT_F32.

    Returns:
        idx: (P, kmax, 2) int32 tensor holding uint32 keypoint indices, rows [0, count) valid per pair.
        count: (P,) int32.
    """
    assert desc.is_cuda and desc.dtype == torch.float32 and desc.dim() == 3 and desc.is_contiguous()
    assert counts.dtype == torch.int32 and pairs.dtype == torch.int32 and pairs.is_contiguous()
    n_img, kmax, dim = desc.shape
    n_pairs = pairs.shape[0]
    L = native.lib()
    idx = torch.empty((max(n_pairs, 1), kmax, 2), dtype=torch.int32, device=desc.device)
    cnt = torch.zeros((max(n_pairs, 1),), dtype=torch.int32, device=desc.device)
    if n_pairs == 0:
        return idx[:0], cnt[:0]
    ws_bytes = L.gtsfm_match_workspace_bytes(n_img, kmax, dim, n_pairs, mode)
    ws = _workspace(ws_bytes, desc.device)
    if stream is not None:
        ws.record_stream(stream)  # the kernels may still read it after this function returns
    rc = L.gtsfm_match_batched(_ptr(desc), _ptr(counts), n_img, kmax, dim, _ptr(pairs), n_pairs,
                               -1.0 if ratio is None else float(ratio), mode, _ptr(ws), ws.numel(), _ptr(idx),
                               _ptr(cnt), native.stream_handle(stream))
    native.check(rc, "gtsfm_match_batched")
    return idx, cnt

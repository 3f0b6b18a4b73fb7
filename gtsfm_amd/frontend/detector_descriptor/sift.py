"""SIFT detector-descriptor on the MI355X.

Drop-in for gtsfm/frontend/detector_descriptor/sift.py:24-56 (SIFTDetectorDescriptor): RGB -> gray
(cv.COLOR_RGB2GRAY fixed point), SIFT with OpenCV's defaults, keypoints (coordinates float64 (N,2), scales = size,
responses), then top-`max_keypoints` by response. Runs in libgtsfm_hip.so (gtsfm_sift_batched); the arithmetic is
the one restated in oracle/sift.c, which reproduces the reference's OpenCV fixture.

The reference's get_top_k order is np.argpartition's (implementation-defined); here keypoints come in descending
response order with a deterministic tie-break.

Image masks follow detectAndCompute(gray, image.mask) (sift.py:47): a keypoint whose rounded pixel is 0 in the mask
is dropped before the top-k. Batches are split so that one launch's workspace stays under WORKSPACE_BUDGET bytes
(the SIFT pyramid costs ~128 B per input pixel).
"""
from typing import Dict, List, Tuple

import numpy as np
import torch

from gtsfm_amd import device, native
from gtsfm_amd.common.image import Image
from gtsfm_amd.common.keypoints import Keypoints
from gtsfm_amd.frontend.detector_descriptor.detector_descriptor_base import DetectorDescriptorBase


def _to_device_batch(arrays: List[np.ndarray]) -> torch.Tensor:
    x = np.ascontiguousarray(np.stack(arrays), dtype=np.uint8)
    if x.ndim == 4 and x.shape[3] == 4:  # RGBA -> RGB (COLOR_RGBA2GRAY uses the same weights)
        x = np.ascontiguousarray(x[..., :3])
    return torch.from_numpy(x).to(torch.device("cuda"))


WORKSPACE_BUDGET = 24 << 30  # bytes of SIFT workspace per launch sequence


def _mask_array(image: Image):
    if image.mask is None:
        return None
    m = np.asarray(image.mask)
    if m.shape != image.value_array.shape[:2]:
        raise ValueError(f"mask shape {m.shape} does not match the image {image.value_array.shape[:2]}")
    return (m != 0).astype(np.uint8)


def sift_groups(images: List[Image], max_kpts: int) -> List[List[int]]:
    """Indices of the images that share one launch: same shape, all masked or none, workspace under budget."""
    by_key: Dict[tuple, List[int]] = {}
    for i, im in enumerate(images):
        by_key.setdefault((im.value_array.shape, im.mask is not None), []).append(i)
    groups: List[List[int]] = []
    L = native.lib()
    for (shape, _), idx in by_key.items():
        per = max(1, int(L.gtsfm_sift_workspace_bytes(1, shape[0], shape[1], max_kpts)))
        n = max(1, WORKSPACE_BUDGET // per)
        groups.extend(idx[s: s + n] for s in range(0, len(idx), n))
    return groups


def extract_group(images: List[Image], idx: List[int], max_kpts: int) -> device.SiftResult:
    """One gtsfm_sift_batched launch sequence over images[idx] (same shape; masks all present or all absent)."""
    masks = None
    if images[idx[0]].mask is not None:
        masks = torch.from_numpy(np.ascontiguousarray(np.stack([_mask_array(images[i]) for i in idx]))).cuda()
    return device.sift_extract(_to_device_batch([images[i].value_array for i in idx]), max_kpts, masks=masks)


def keypoints_from_result(res: device.SiftResult, i: int) -> Tuple[Keypoints, np.ndarray]:
    n = int(res.count[i].item())
    xy = res.xy[i, :n].cpu().numpy().astype(np.float64)
    attr = res.attr[i, :n].cpu().numpy().astype(np.float64)
    desc = res.desc[i, :n].cpu().numpy()
    return Keypoints(coordinates=xy, scales=attr[:, 0], responses=attr[:, 2]), desc


class SIFTDetectorDescriptor(DetectorDescriptorBase):
    """SIFT detector-descriptor computed by HIP kernels."""

    def detect_and_describe(self, image: Image) -> Tuple[Keypoints, np.ndarray]:
        native.require_gpu()
        return keypoints_from_result(extract_group([image], [0], self.max_keypoints), 0)

    def detect_and_describe_batch(self, images: List[Image]) -> List[Tuple[Keypoints, np.ndarray]]:
        """Images of one size in batched launch sequences (sift_groups)."""
        native.require_gpu()
        out: List[Tuple[Keypoints, np.ndarray]] = [None] * len(images)  # type: ignore
        for idx in sift_groups(images, self.max_keypoints):
            res = extract_group(images, idx, self.max_keypoints)
            for j, i in enumerate(idx):
                out[i] = keypoints_from_result(res, j)
        return out

"""SIFT detector-descriptor on the MI355X.

Drop-in for gtsfm/frontend/detector_descriptor/sift.py:24-56 (SIFTDetectorDescriptor): RGB -> gray
(cv.COLOR_RGB2GRAY fixed point), SIFT with OpenCV's defaults, keypoints (coordinates float64 (N,2), scales = size,
responses), then top-`max_keypoints` by response. Runs in libgtsfm_hip.so (gtsfm_sift_batched); the arithmetic is
the one restated in oracle/sift.c, which reproduces the reference's OpenCV fixture.

The reference's get_top_k order is np.argpartition's (implementation-defined); here keypoints come in descending
response order with a deterministic tie-break.
"""
from typing import List, Tuple

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
        if image.mask is not None:
            raise NotImplementedError("SIFT masks are not supported on the MI355X path yet")
        res = device.sift_extract(_to_device_batch([image.value_array]), self.max_keypoints)
        return keypoints_from_result(res, 0)

    def detect_and_describe_batch(self, images: List[Image]) -> List[Tuple[Keypoints, np.ndarray]]:
        """All images of one size in a single batched launch sequence."""
        native.require_gpu()
        out: List[Tuple[Keypoints, np.ndarray]] = [None] * len(images)  # type: ignore
        by_shape = {}
        for i, im in enumerate(images):
            by_shape.setdefault(im.value_array.shape, []).append(i)
        for _, idx in by_shape.items():
            res = device.sift_extract(_to_device_batch([images[i].value_array for i in idx]), self.max_keypoints)
            for j, i in enumerate(idx):
                out[i] = keypoints_from_result(res, j)
        return out

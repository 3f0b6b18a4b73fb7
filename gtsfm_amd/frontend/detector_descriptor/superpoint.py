"""SuperPoint detector-descriptor on the MI355X.

Drop-in for gtsfm/frontend/detector_descriptor/superpoint.py:28-74 (SuperPointDetectorDescriptor): same constructor
(max_keypoints, use_cuda, weights_path), same outputs: Keypoints(coordinates (N,2) float32 (x, y), scales=None,
responses=scores) and (N, 256) float32 unit descriptors, top-`max_keypoints` by score. The network
(thirdparty/SuperGluePretrainedNetwork/models/superpoint.py:145-202: encoder, score head + simple_nms, descriptor
head + bilinear sampling) runs in libgtsfm_hip.so (gtsfm_superpoint_batched) on the fp32 matrix cores.

Weights: a torch state dict with the reference module's parameter names, loaded with torch.load(weights_only=True)
from `weights_path` (superpoint_v1.pth), or passed in directly as `state_dict` (name -> array).
"""
from pathlib import Path
from typing import Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from gtsfm_amd import device, native
from gtsfm_amd.common.image import Image
from gtsfm_amd.common.keypoints import Keypoints
from gtsfm_amd.frontend.detector_descriptor.detector_descriptor_base import DetectorDescriptorBase

MODEL_WEIGHTS_PATH = Path("thirdparty/SuperGluePretrainedNetwork/models/weights/superpoint_v1.pth")

# (name(s), k, cin, cout_pad): the packed blob layout of include/gtsfm_hip.h
_PACK = [(("conv1a",), 3, 1, 64), (("conv1b",), 3, 64, 64), (("conv2a",), 3, 64, 64), (("conv2b",), 3, 64, 64),
         (("conv3a",), 3, 64, 128), (("conv3b",), 3, 128, 128), (("conv4a",), 3, 128, 128),
         (("conv4b",), 3, 128, 128), (("convPa", "convDa"), 3, 128, 512), (("convPb",), 1, 256, 128),
         (("convDb",), 1, 256, 256)]


def pack_superpoint_weights(state_dict: Dict[str, np.ndarray]) -> np.ndarray:
    """Reference state dict (name.weight (cout, cin, k, k), name.bias) -> the packed fp32 blob."""
    parts = []
    for names, k, cin, cout_pad in _PACK:
        w = np.concatenate([np.asarray(state_dict[f"{nm}.weight"], np.float32) for nm in names], axis=0)
        b = np.concatenate([np.asarray(state_dict[f"{nm}.bias"], np.float32) for nm in names], axis=0)
        cout = w.shape[0]
        assert w.shape == (cout, cin, k, k), (names, w.shape)
        wp = np.zeros((k * k, cin, cout_pad), np.float32)
        wp[:, :, :cout] = w.transpose(2, 3, 1, 0).reshape(k * k, cin, cout)
        bp = np.zeros(cout_pad, np.float32)
        bp[:cout] = b
        parts += [wp.ravel(), bp]
    return np.concatenate(parts)


def load_state_dict(weights_path: Union[Path, str]) -> Dict[str, np.ndarray]:
    sd = torch.load(str(weights_path), map_location="cpu", weights_only=True)
    return {k: v.numpy() for k, v in sd.items()}


class SuperPointDetectorDescriptor(DetectorDescriptorBase):
    """SuperPoint computed by HIP kernels (keypoint_threshold 0.005, nms_radius 4, remove_borders 4 as the
    reference module's default_config)."""

    def __init__(self, max_keypoints: int = 5000, use_cuda: bool = True,
                 weights_path: Union[Path, str] = MODEL_WEIGHTS_PATH,
                 state_dict: Optional[Dict[str, np.ndarray]] = None, keypoint_threshold: float = 0.005,
                 nms_radius: int = 4, remove_borders: int = 4) -> None:
        super().__init__(max_keypoints=max_keypoints)
        self._use_cuda = use_cuda
        self._config = {"weights_path": weights_path}
        self._state_dict = state_dict
        self._blob: Optional[torch.Tensor] = None
        self._thr, self._nms, self._border = keypoint_threshold, nms_radius, remove_borders

    def __getstate__(self):
        s = self.__dict__.copy()
        s["_blob"] = None  # device memory is re-created per process
        return s

    def weights(self) -> torch.Tensor:
        if self._blob is None:
            native.require_gpu()
            sd = self._state_dict if self._state_dict is not None else load_state_dict(self._config["weights_path"])
            self._blob = torch.from_numpy(pack_superpoint_weights(sd)).to(torch.device("cuda"))
        return self._blob

    def extract_batch(self, arrays: List[np.ndarray], max_kpts: Optional[int] = None,
                      masks: Optional[List[Optional[np.ndarray]]] = None) -> device.SuperPointResult:
        """Same-sized images; masks: per image an (H, W) array (keypoints kept where it equals 1, as the reference's
        Keypoints.filter_by_mask before get_top_k) or None (all kept)."""
        x = np.ascontiguousarray(np.stack(arrays), dtype=np.uint8)
        if x.ndim == 4 and x.shape[3] == 4:
            x = np.ascontiguousarray(x[..., :3])
        dev = torch.device("cuda")
        t = torch.from_numpy(x).to(dev)
        m = None
        if masks is not None and any(mk is not None for mk in masks):
            H, W = x.shape[1], x.shape[2]
            mm = np.ones((len(arrays), H, W), np.uint8)
            for i, mk in enumerate(masks):
                if mk is not None:
                    mk = np.asarray(mk)
                    assert mk.shape[:2] == (H, W), (mk.shape, (H, W))
                    mm[i] = mk.reshape(H, W) == 1  # filter_by_mask's test, as 0 / 1 bytes
            m = torch.from_numpy(mm).to(dev)
        return device.superpoint_extract(t, self.weights(), max_kpts or self.max_keypoints, self._thr, self._nms,
                                         self._border, masks=m)

    @staticmethod
    def _unpack(res: device.SuperPointResult, i: int) -> Tuple[Keypoints, np.ndarray]:
        n = int(res.count[i].item())
        xy = res.xy[i, :n].cpu().numpy()
        scores = res.scores[i, :n].cpu().numpy()
        desc = res.desc[i, :n].cpu().numpy()
        return Keypoints(coordinates=xy, scales=None, responses=scores), desc

    def detect_and_describe(self, image: Image) -> Tuple[Keypoints, np.ndarray]:
        """Reference superpoint.py:48-74: network, then filter_by_mask(image.mask) when given, then
        get_top_k(max_keypoints), all on the device."""
        native.require_gpu()
        return self._unpack(self.extract_batch([image.value_array], masks=[image.mask]), 0)

    def detect_and_describe_batch(self, images: List[Image]) -> List[Tuple[Keypoints, np.ndarray]]:
        native.require_gpu()
        out: List[Tuple[Keypoints, np.ndarray]] = [None] * len(images)  # type: ignore
        by_shape: Dict[tuple, List[int]] = {}
        for i, im in enumerate(images):
            by_shape.setdefault(im.value_array.shape, []).append(i)
        for _, idx in by_shape.items():
            res = self.extract_batch([images[i].value_array for i in idx], masks=[images[i].mask for i in idx])
            for j, i in enumerate(idx):
                out[i] = self._unpack(res, j)
        return out

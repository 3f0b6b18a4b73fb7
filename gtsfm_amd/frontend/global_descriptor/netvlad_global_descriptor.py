"""NetVLAD global image descriptor on the MI355X.

Drop-in for gtsfm/frontend/global_descriptor/netvlad_global_descriptor.py:20-46 (NetVLADGlobalDescriptor) and the
network it runs, thirdparty/hloc/netvlad.py:74-191 (VGG16-NetVLAD with whitening): same `describe(image)` -> (4096,)
float32 unit vector for an RGB image. The whole network runs in libgtsfm_hip.so (gtsfm_netvlad_batched, netvlad.hip):
the VGG16 backbone on the bf16 matrix cores at fp32 accuracy, the VLAD layer and the whitening as fp32 MFMA GEMMs.
`describe_batch` / `describe_device` run every image of one size in one launch sequence and can leave the
descriptors in HBM for the retriever (gtsfm_amd/retriever/image_pairs_generator.py).

Weights: the reference's checkpoint (VGG16-NetVLAD-Pitts30K.mat, which netvlad.py downloads; absent offline) parsed
exactly as NetVLAD.__init__ does (netvlad.py:112-152: backbone conv layers from mat["net"].layers, score_proj from
layer 30, negated centres, whitening from layer 33, averageImage as the mean), or a state dict under the reference
module's parameter names (backbone.{i}.weight/bias, netvlad.score_proj.weight, netvlad.centers, whiten.weight/bias)
plus "preprocess_mean". The reference rebuilds the model on every describe() call (its note: constructing it in
__init__ ran out of memory); here the packed weights are built once per process and kept on the device.
"""
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from gtsfm_amd import device, native
from gtsfm_amd.common.image import Image
from gtsfm_amd.frontend.global_descriptor.global_descriptor_base import GlobalDescriptorBase

# thirdparty/hloc/netvlad.py:23 + default_conf (:75): {checkpoint_dir}/VGG16-NetVLAD-Pitts30K.mat
CHECKPOINT_PATH = Path("thirdparty/hloc/weights/VGG16-NetVLAD-Pitts30K.mat")
VGG16_CONV_INDICES = (0, 2, 5, 7, 10, 12, 14, 17, 19, 21, 24, 26, 28)  # conv children of VGG16 features[:-2]
VGG16_CHANNELS = ((3, 64), (64, 64), (64, 128), (128, 128), (128, 256), (256, 256), (256, 256), (256, 512),
                  (512, 512), (512, 512), (512, 512), (512, 512), (512, 512))
DIM, CLUSTERS, WHITE_DIM = 512, 64, 4096
WORKSPACE_BUDGET = 32 << 30  # bytes of workspace per launch sequence (~1.1 KB per input pixel)


def load_netvlad_mat(path: Union[str, Path]) -> Dict[str, np.ndarray]:
    """The reference checkpoint -> state dict, as NetVLAD.__init__ maps it (netvlad.py:112-152)."""
    import scipy.io

    mat = scipy.io.loadmat(str(path), struct_as_record=False, squeeze_me=True)
    layers = mat["net"].layers
    sd: Dict[str, np.ndarray] = {}
    for idx in VGG16_CONV_INDICES:
        w, b = layers[idx].weights[0], layers[idx].weights[1]  # S x S x IN x OUT, OUT
        sd[f"backbone.{idx}.weight"] = np.ascontiguousarray(np.asarray(w, np.float32).transpose(3, 2, 0, 1))
        sd[f"backbone.{idx}.bias"] = np.asarray(b, np.float32).reshape(-1)
    sd["netvlad.score_proj.weight"] = np.asarray(layers[30].weights[0], np.float32).T[:, :, None]  # K x D x 1
    sd["netvlad.centers"] = -np.asarray(layers[30].weights[1], np.float32)  # stored negated (:140-141)
    ww = np.asarray(layers[33].weights[0], np.float32)
    sd["whiten.weight"] = np.ascontiguousarray(ww.reshape(ww.shape[-2], ww.shape[-1]).T)  # OUT x IN
    sd["whiten.bias"] = np.asarray(layers[33].weights[1], np.float32).reshape(-1)
    sd["preprocess_mean"] = np.asarray(mat["net"].meta.normalization.averageImage, np.float32).reshape(-1)[:3]
    return sd


def pack_netvlad_weights(state_dict: Dict[str, np.ndarray]) -> np.ndarray:
    """State dict -> the packed fp32 blob of include/gtsfm_hip.h (gtsfm_netvlad_batched)."""
    parts = [np.concatenate([np.asarray(state_dict["preprocess_mean"], np.float32).reshape(3), np.zeros(1, np.float32)])]
    for idx, (cin, cout) in zip(VGG16_CONV_INDICES, VGG16_CHANNELS):
        w = np.asarray(state_dict[f"backbone.{idx}.weight"], np.float32)
        assert w.shape == (cout, cin, 3, 3), (idx, w.shape)
        parts += [w.transpose(2, 3, 1, 0).reshape(-1), np.asarray(state_dict[f"backbone.{idx}.bias"], np.float32)]
    score = np.asarray(state_dict["netvlad.score_proj.weight"], np.float32).reshape(CLUSTERS, DIM)
    centers = np.asarray(state_dict["netvlad.centers"], np.float32).reshape(DIM, CLUSTERS)
    parts += [score.reshape(-1), centers.reshape(-1)]
    if "whiten.weight" in state_dict:
        ww = np.asarray(state_dict["whiten.weight"], np.float32)
        assert ww.shape == (WHITE_DIM, DIM * CLUSTERS), ww.shape
        parts += [ww.reshape(-1), np.asarray(state_dict["whiten.bias"], np.float32).reshape(WHITE_DIM)]
    else:  # conf["whiten"] False: the whitening slots are unused
        parts += [np.zeros(WHITE_DIM * DIM * CLUSTERS + WHITE_DIM, np.float32)]
    return np.concatenate(parts)


class NetVLADGlobalDescriptor(GlobalDescriptorBase):
    """NetVLAD (VGG16 + NetVLAD layer + whitening) computed by HIP kernels."""

    def __init__(self, checkpoint_path: Union[str, Path] = CHECKPOINT_PATH,
                 state_dict: Optional[Dict[str, np.ndarray]] = None, whiten: bool = True) -> None:
        self._checkpoint_path = Path(checkpoint_path)
        self._state_dict = state_dict
        self._whiten = whiten
        self._blob: Optional[torch.Tensor] = None

    def __repr__(self) -> str:
        return f"NetVLADGlobalDescriptor(whiten={self._whiten})"

    def __getstate__(self):
        s = self.__dict__.copy()
        s["_blob"] = None  # device memory is re-created per process
        return s

    def weights(self) -> torch.Tensor:
        if self._blob is None:
            native.require_gpu()
            sd = self._state_dict if self._state_dict is not None else load_netvlad_mat(self._checkpoint_path)
            self._blob = torch.from_numpy(pack_netvlad_weights(sd)).to(torch.device("cuda"))
        return self._blob

    def describe_device(self, images: Sequence[Image]) -> torch.Tensor:
        """(n, 4096) f32 device tensor (n, 32768 without whitening): images grouped by size, each group in
        workspace-bounded launch sequences of gtsfm_netvlad_batched."""
        native.require_gpu()
        dev = torch.device("cuda")
        dim = WHITE_DIM if self._whiten else DIM * CLUSTERS
        out = torch.empty((len(images), dim), dtype=torch.float32, device=dev)
        by_shape: Dict[tuple, List[int]] = {}
        for i, im in enumerate(images):
            a = im.value_array
            if a.ndim != 3 or a.shape[2] != 3:
                raise ValueError(f"NetVLAD needs an (H, W, 3) RGB image, got {a.shape} (netvlad.py:172)")
            by_shape.setdefault(a.shape, []).append(i)
        L = native.lib()
        w = self.weights()
        for shape, idx in by_shape.items():
            per = max(1, int(L.gtsfm_netvlad_workspace_bytes(1, shape[0], shape[1])))
            g = max(1, WORKSPACE_BUDGET // per)
            for s in range(0, len(idx), g):
                part = idx[s: s + g]
                x = torch.from_numpy(np.ascontiguousarray(np.stack([images[i].value_array for i in part]),
                                                          dtype=np.uint8)).to(dev)
                desc, vlad = device.netvlad_describe(x, w, whiten=self._whiten)
                out[torch.tensor(part, dtype=torch.long, device=dev)] = desc if self._whiten else vlad
        return out

    def describe_batch(self, images: List[Image]) -> List[np.ndarray]:
        d = self.describe_device(images).cpu().numpy()
        return [d[i].copy() for i in range(len(images))]

    def describe(self, image: Image) -> np.ndarray:
        """netvlad_global_descriptor.py:27-46: (4096,) float32 descriptor of one image."""
        return self.describe_device([image])[0].cpu().numpy()

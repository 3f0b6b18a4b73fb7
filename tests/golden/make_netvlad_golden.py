"""Golden NetVLAD global descriptors from the reference's own module (run in the build container, where /root/reference
exists; the GPU box has no reference and only reads the .npz this writes).

thirdparty/hloc/netvlad.py is imported as-is with `torchvision` stubbed in sys.modules: the module imports it only
for `models.vgg16()` inside NetVLAD.__init__ (netvlad.py:108), which also downloads and parses the .mat checkpoint
(absent offline). The model is therefore assembled without running __init__:
- backbone: VGG16 `features[:-2]` as an nn.Sequential built here from torchvision's published configuration "D"
  (the layer list netvlad.py:108-110 obtains from torchvision) -- parity of this list is UNPINNED (torchvision is
  absent), its arithmetic is plain torch conv2d / relu / max_pool2d;
- netvlad: the reference's NetVLADLayer class itself (netvlad.py:28-71);
- whiten: nn.Linear(32768, 4096) (netvlad.py:118-119);
- preprocess: {"mean": ..., "std": [1, 1, 1]} (netvlad.py:149-152);
and NetVLAD.forward (netvlad.py:160-191) -- clamp/scale, mean subtraction, backbone, pre-normalisation, VLAD,
whitening, final L2 -- runs unmodified, on the input NetVLADGlobalDescriptor.describe builds
(netvlad_global_descriptor.py:36-46: u8 HWC -> CHW float / 255). Weights: tests/netvlad_weights.py (seed 0).

Recorded per case: the 4096-D descriptor and the 32768-D VLAD vector (NetVLADLayer's output, via a forward hook).

    python tests/golden/make_netvlad_golden.py
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, REF)
sys.path.insert(0, os.path.dirname(HERE))  # tests/

from netvlad_weights import VGG16_CONVS, netvlad_cases as cases, netvlad_state_dict  # noqa: E402


def vgg16_features_minus_2() -> nn.Sequential:
    layers = []
    for _, cin, cout, pool in VGG16_CONVS:
        layers += [nn.Conv2d(cin, cout, 3, padding=1), nn.ReLU(inplace=True)]
        if pool:
            layers.append(nn.MaxPool2d(2, 2))
    return nn.Sequential(*layers[:-1])  # features[:-2]: the last ReLU and MaxPool2d removed (pool already absent)


def reference_netvlad(seed=0):
    tv = types.ModuleType("torchvision")
    tv.models = types.ModuleType("torchvision.models")
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.models", tv.models)
    from thirdparty.hloc import netvlad as nv

    sd = netvlad_state_dict(seed)
    model = nv.NetVLAD.__new__(nv.NetVLAD)
    nn.Module.__init__(model)
    model.backbone = vgg16_features_minus_2()
    model.netvlad = nv.NetVLADLayer()
    model.whiten = nn.Linear(model.netvlad.output_dim, 4096)
    for name, p in model.named_parameters():
        p.data = torch.from_numpy(sd[name].copy())
    model.preprocess = {"mean": sd["preprocess_mean"], "std": np.array([1, 1, 1], dtype=np.float32)}
    return model.eval()


def main():
    torch.set_num_threads(8)
    model = reference_netvlad(0)
    vlad = {}
    model.netvlad.register_forward_hook(lambda m, i, o: vlad.__setitem__("v", o.detach().clone()))
    res = {}
    for name, imgs in cases().items():
        descs, vlads = [], []
        for im in imgs:
            x = torch.from_numpy(im).permute(2, 0, 1).unsqueeze(0).type(torch.float32) / 255  # describe() (:40-42)
            with torch.no_grad():
                d = model({"image": x})["global_descriptor"]
            descs.append(d[0].numpy())
            vlads.append(vlad["v"][0].numpy())
        res[f"{name}/desc"] = np.stack(descs).astype(np.float32)
        res[f"{name}/vlad"] = np.stack(vlads).astype(np.float32)
        print(name, res[f"{name}/desc"].shape, float(np.abs(res[f"{name}/desc"]).max()))
    np.savez_compressed(os.path.join(HERE, "netvlad_random_w0.npz"), **res)


if __name__ == "__main__":
    main()

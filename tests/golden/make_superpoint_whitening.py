"""Whitened descriptor head for the seeded random SuperPoint weights (bench / test data, not a reference output).

With random weights (tests/superpoint_weights.superpoint_state_dict) the 256-D SuperPoint descriptors of a scene are
almost parallel (mean cosine 0.99 between unrelated keypoints), so neither SuperGlue nor the F16_RERANK matcher sees a
realistic descriptor distribution: SuperGlue matches nothing and the fp16 shortlist cannot certify. This script keeps
the seeded encoder and descriptor layer convDa and replaces the 1x1 layer convDb by the ZCA whitening of convDa's
activations over four rendered 1080p views of the benchmark scene (synthetic.render_scene, views 0/8/16/24 of a
32-camera orbit): W = C^-1/2, b = -W mu. Descriptors of unrelated keypoints then have cosine ~0 and repeated scene
points match (mutual nearest neighbours of adjacent views are ~35 % geometrically consistent at 4 px). The result is
stored as tests/golden/superpoint_w0_convDb_whitened.npz and used by
tests/superpoint_weights.superpoint_state_dict(0, whitened=True) for BASELINE configs C3 / C5 in bench.py and the C5
GPU test. Generated with the CPU restatement oracle/deep.py.

    python tests/golden/make_superpoint_whitening.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(HERE))

from superpoint_weights import superpoint_state_dict  # noqa: E402

VIEWS = (0, 8, 16, 24)
ORBIT = 32


def main():
    from gtsfm_amd import synthetic
    from oracle import deep, oracle

    torch.set_num_threads(8)
    sd = superpoint_state_dict(0)
    scene = synthetic.render_scene(ORBIT, 1080, 1920, device="cpu", indices=list(VIEWS))
    feats = []
    for j in range(len(VIEWS)):
        gray = oracle.rgb_to_gray(scene.images[j].numpy())
        with torch.no_grad():
            x = deep.superpoint_encoder(gray, sd)
            a = deep._conv(x, sd, "convDa")[0]
        feats.append(a.reshape(a.shape[0], -1).T.double())
        print("view", VIEWS[j], tuple(a.shape), flush=True)
    A = torch.cat(feats)
    mu = A.mean(0)
    C = torch.cov(A.T)
    ev, V = torch.linalg.eigh(C)
    Wz = V @ torch.diag(1.0 / torch.sqrt(ev.clamp_min(1e-6 * float(ev.max())))) @ V.T
    np.savez_compressed(os.path.join(HERE, "superpoint_w0_convDb_whitened.npz"),
                        weight=Wz.float().numpy()[:, :, None, None], bias=(-(Wz @ mu)).float().numpy(),
                        views=np.array(VIEWS), orbit=np.array(ORBIT))
    print("wrote superpoint_w0_convDb_whitened.npz")


if __name__ == "__main__":
    main()

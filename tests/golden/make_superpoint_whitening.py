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

    python tests/golden/make_superpoint_whitening.py          # C5 head (ZCA, orbit scene)
    python tests/golden/make_superpoint_whitening.py --c3     # C3 head (see below)

--c3 writes tests/golden/superpoint_w0_convDb_pca32_strafe.npz for BASELINE config C3 (SuperPoint + TwoWayMatcher
mutual NN + ratio 0.8): fitted on views 0 / 100 / 199 of the 200-camera "strafe" path of synthetic.render_scene; the
32 leading principal directions of convDa's activations are whitened and the remaining ones whitened at a quarter
weight (W = V_32 diag(ev_32^-1/2) V_32^T + 0.25 V_r diag(ev_r^-1/2) V_r^T, b = -W mu). The trailing directions of a
random encoder mostly carry view-dependent aliasing of its stride-2 pools: at full weight (the ZCA head) mutual NN +
the ratio test keep ~30 matches per pair of that scene; dropped entirely (rank 32) ~300, but the descriptors are then
so clustered that F16_RERANK's fp16 shortlist rarely certifies (matching 4.5 s instead of 0.75 s per C3 step); at a
quarter weight ~185 putatives per pair, 95 % of the pairs verified, and the matcher certifies as with trained-like
descriptors (measured on the GPU bench, bench.py --config c3).
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

    c3 = "--c3" in sys.argv[1:]
    torch.set_num_threads(8)
    sd = superpoint_state_dict(0)
    views, n_cam = ((0, 100, 199), 200) if c3 else (VIEWS, ORBIT)
    scene = synthetic.render_scene(n_cam, 1080, 1920, device="cpu", indices=list(views),
                                   path="strafe" if c3 else "orbit")
    feats = []
    for j in range(len(views)):
        gray = oracle.rgb_to_gray(scene.images[j].numpy())
        with torch.no_grad():
            x = deep.superpoint_encoder(gray, sd)
            a = deep._conv(x, sd, "convDa")[0]
        feats.append(a.reshape(a.shape[0], -1).T.double())
        print("view", views[j], tuple(a.shape), flush=True)
    A = torch.cat(feats)
    mu = A.mean(0)
    C = torch.cov(A.T)
    ev, V = torch.linalg.eigh(C)
    if c3:
        V32, e32 = V[:, -32:], ev[-32:]
        Vr, er = V[:, :-32], ev[:-32].clamp_min(1e-6 * float(ev.max()))
        Wz = V32 @ torch.diag(1.0 / torch.sqrt(e32)) @ V32.T + 0.25 * (Vr @ torch.diag(1.0 / torch.sqrt(er)) @ Vr.T)
        name = "superpoint_w0_convDb_pca32_strafe.npz"
    else:
        Wz = V @ torch.diag(1.0 / torch.sqrt(ev.clamp_min(1e-6 * float(ev.max())))) @ V.T
        name = "superpoint_w0_convDb_whitened.npz"
    np.savez_compressed(os.path.join(HERE, name), weight=Wz.float().numpy()[:, :, None, None],
                        bias=(-(Wz @ mu)).float().numpy(), views=np.array(views), orbit=np.array(n_cam))
    print("wrote", name)


if __name__ == "__main__":
    main()

"""GPU vs oracle SIFT detections on the Lund image: the keypoints only one side has (debug helper)."""
import os
import sys

import numpy as np
import torch
from PIL import Image as PILImage

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from gtsfm_amd import device  # noqa: E402
from oracle import oracle  # noqa: E402

gray = np.asarray(PILImage.open(os.path.join(REPO, "tests/golden/lund_door_DSC_0001_gray.png")))
k = 8192
res = device.sift_extract(torch.from_numpy(np.ascontiguousarray(gray)[None]).cuda(), k)
n = int(res.count[0])
kp = np.concatenate([res.xy[0, :n].cpu().numpy(), res.attr[0, :n].cpu().numpy()], 1)
rkp, _, rnd = oracle.sift(gray, k)
print("gpu", n, int(res.n_detected[0]), "oracle", len(rkp), rnd, gray.shape)
a = {tuple(np.round(r[:2], 4)) for r in kp}
b = {tuple(np.round(r[:2], 4)) for r in rkp}
extra = [r for r in kp if tuple(np.round(r[:2], 4)) not in b]
miss = [r for r in rkp if tuple(np.round(r[:2], 4)) not in a]
print("gpu-only", len(extra), "oracle-only", len(miss))
for name, rows in (("gpu-only", extra), ("oracle-only", miss)):
    for r in rows[:40]:
        size = r[2]
        print(name, "x %.2f y %.2f size %.2f  x2 mod 64 %.1f" % (r[0], r[1], size, (2 * r[0]) % 64))

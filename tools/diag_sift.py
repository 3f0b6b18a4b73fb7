"""Diagnostic: SIFT run-to-run and batch-composition determinism on the bench scene (valid rows only)."""
import os, sys
import numpy as np, torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from gtsfm_amd import device as hip, synthetic
n = 100
scene = synthetic.render_scene(n, 1080, 1920, device="cuda")
imgs = scene.images
runs = [hip.sift_extract(imgs, 2048) for _ in range(2)]
half = [hip.sift_extract(imgs[:50].contiguous(), 2048), hip.sift_extract(imgs[50:].contiguous(), 2048)]
torch.cuda.synchronize()
def get(r):
    return {k: getattr(r, k).cpu().numpy() for k in ("xy", "attr", "desc", "count", "n_detected")}
A, B = get(runs[0]), get(runs[1])
H = {k: np.concatenate([getattr(half[0], k).cpu().numpy(), getattr(half[1], k).cpu().numpy()]) for k in A}
def cmp(X, Y, tag):
    bad = []
    for i in range(n):
        c = X["count"][i]
        if c != Y["count"][i] or X["n_detected"][i] != Y["n_detected"][i]:
            bad.append((i, "count", int(c), int(Y["count"][i]))); continue
        for k in ("xy", "attr", "desc"):
            d = np.nonzero((X[k][i, :c] != Y[k][i, :c]).reshape(c, -1).any(1))[0]
            if len(d):
                r = d[0]
                bad.append((i, k, len(d), int(r), X["xy"][i, r].tolist(), X["attr"][i, r].tolist(), Y["attr"][i, r].tolist()))
    print(tag, "images differing:", len(set(b[0] for b in bad)))
    for b in bad[:12]:
        print("  ", b)
cmp(A, B, "run-to-run")
cmp(A, H, "full-vs-halves")

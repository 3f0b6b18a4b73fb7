"""BASELINE config C1 fixtures: the reference's 12 Lund Door images + ground truth, and the oracle's front-end results
on all 66 pairs (run in the build container, where /root/reference exists).

Data taken from the reference (tests/data/set1_lund_door/): the 12 JPEGs, copied byte for byte into
tests/golden/lund_door/ (decoded on the GPU box with PIL, as the reference's loader does: gtsfm/utils/io.py:40-53),
and the 3x4 projection matrices of data.mat, decomposed as OlssonLoader does (olsson_loader.py:66-91,
verification.py:20-49: RQ with positive diagonal; intrinsics fx = min(K00, K11), u0 = K02, v0 = K12,
olsson_loader.py:126-147) into lund_door/gt.json.

Expected outputs come from the CPU oracle, run with sift_front_end.yaml's parameters at max_resolution 1296 (the
reference CI benchmark's setting, .github/workflows/benchmark.yml; the 1296 x 1936 images need no resize):
SIFT max_keypoints 5000 -> TwoWayMatcher ratio 0.8 -> Ransac(use_intrinsics_in_verification=True,
estimation_threshold_px=4; MSAC model selection, USAC_ACCURATE's scoring) with the sampler stream of one verify()
call per pair (pair id 0).
Stored: keypoint counts and sha256 of each image's (xy, descriptors), every pair's putatives, and the verifier's
status / inlier count / R / t.

    python tests/golden/make_lund_c1_golden.py
"""
import hashlib
import json
import os
import shutil
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/tests/data/set1_lund_door"
OUT = os.path.join(HERE, "lund_door")
sys.path.insert(0, REPO)

MAX_KPTS, RATIO, THR_PX = 5000, 0.8, 4.0


def decompose(M):
    import scipy.linalg

    Q, m4 = M[:3, :3], M[:, 3]
    wtc = np.linalg.inv(-Q) @ m4
    K, cRw = scipy.linalg.rq(Q)
    T = np.diag(np.sign(np.diag(K)))
    K = K @ T
    wRc = (T @ cRw).T
    return K, wRc, wtc


def load_rgb(path):
    from PIL import Image

    return np.asarray(Image.open(path).convert("RGB"))


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    import scipy.io

    from oracle import oracle

    os.makedirs(OUT, exist_ok=True)
    names = sorted(f for f in os.listdir(os.path.join(REF, "images")) if f.endswith(".JPG"))
    assert len(names) == 12
    for n in names:
        shutil.copyfile(os.path.join(REF, "images", n), os.path.join(OUT, n))
    P = scipy.io.loadmat(os.path.join(REF, "data.mat"))["P"][0]
    K0, _, _ = decompose(P[0])
    cams = [decompose(P[i]) for i in range(12)]
    intr = [float(min(K0[0, 0], K0[1, 1])), float(K0[0, 2]), float(K0[1, 2])]
    gt = {"images": names, "fx_u0_v0": intr, "wRc": [c[1].tolist() for c in cams], "wtc": [c[2].tolist() for c in cams],
          "source": "tests/data/set1_lund_door/data.mat P, decomposed as olsson_loader.py:66-91"}
    with open(os.path.join(OUT, "gt.json"), "w") as f:
        json.dump(gt, f, indent=1)

    imgs = [load_rgb(os.path.join(OUT, n)) for n in names]
    f, u0, v0 = intr

    def sift_one(im):
        kp, desc, nd = oracle.sift(oracle.rgb_to_gray(im), MAX_KPTS)
        return kp, desc, nd

    with ThreadPoolExecutor(8) as pool:
        feats = list(pool.map(sift_one, imgs))
    pairs = [(i, j) for i in range(12) for j in range(i + 1, 12)]

    def pair_one(p):
        (k1, d1, _), (k2, d2, _) = feats[p[0]], feats[p[1]]
        m = oracle.twoway_match(d1, d2, RATIO).reshape(-1, 2)
        out = {"m": m, "status": 1, "n": 0, "R": np.zeros((3, 3)), "t": np.zeros(3), "mask": np.zeros(len(m), np.uint8)}
        if len(m) >= 6:
            x1 = (k1[m[:, 0], :2].astype(np.float64) - [u0, v0]) / f
            x2 = (k2[m[:, 1], :2].astype(np.float64) - [u0, v0]) / f
            r = oracle.ransac_E(x1, x2, THR_PX / f, pair_id=0)
            if r is None:
                out["status"] = 2
            else:
                E, mask, R, t, n, nh = r
                out.update(status=0, n=n, R=R, t=t, mask=mask)
        return out

    with ThreadPoolExecutor(8) as pool:
        res = list(pool.map(pair_one, pairs))
    counts = np.array([len(r["m"]) for r in res])
    np.savez_compressed(
        os.path.join(OUT, "oracle_c1.npz"),
        kp_count=np.array([len(x[0]) for x in feats]), n_detected=np.array([x[2] for x in feats]),
        pairs=np.array(pairs), match_count=counts, matches=np.concatenate([r["m"] for r in res]).astype(np.uint32),
        masks=np.concatenate([r["mask"] for r in res]), status=np.array([r["status"] for r in res]),
        n_inliers=np.array([r["n"] for r in res]), R=np.stack([r["R"] for r in res]),
        t=np.stack([r["t"] for r in res]))
    with open(os.path.join(OUT, "oracle_c1_features.json"), "w") as fh:
        json.dump({"sha256_xy_desc": [sha(x[0][:, :2], x[1]) for x in feats],
                   "sha256_kp5_desc": [sha(x[0], x[1]) for x in feats]}, fh, indent=1)
    print("kpts", [len(x[0]) for x in feats])
    print("matches", counts.min(), counts.mean(), counts.max(), "verified", [r["n"] for r in res][:12])


if __name__ == "__main__":
    main()

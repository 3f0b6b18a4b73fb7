"""Generates the committed golden fixtures under tests/golden/ (run in the build container, where
/root/reference exists). Only DATA is taken from the reference: the inputs/expected outputs of its known-answer
tests and slices of its fixture arrays. Expected outputs the reference does not hold are produced by the CPU
oracle (oracle/), which is itself pinned by the reference's known answers (tests/test_oracle.py).

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)


def twoway_known_answers():
    # tests/frontend/matcher/test_twoway_withratiotest_matcher.py:25-49 and
    # tests/frontend/matcher/test_twoway_withoutratiotest_matcher.py:25-46 (inputs and expected matches)
    d1 = [0.4865, 0.3752, 0.3077, 0.9188, 0.7837, 0.1083, 0.6822, 0.3764, 0.2288, 0.8018, 1.1]
    d2 = [0.9995, 0.3376, 0.9005, 0.5382, 0.3162, 0.7974, 0.1785, 0.3491, 0.8658, 0.2912]
    out = {
        "descriptors_i1": d1,
        "descriptors_i2": d2,
        "expected_ratio_0.8": [[9, 5], [2, 4], [3, 2], [0, 3]],
        "expected_no_ratio": [[9, 5], [2, 4], [3, 2], [1, 7], [8, 6], [0, 3]],
        "source": "tests/frontend/matcher/test_twoway_with{,out}ratiotest_matcher.py",
    }
    with open(os.path.join(HERE, "twoway_known_answers.json"), "w") as f:
        json.dump(out, f, indent=1)


def lund_door_descriptors():
    # tests/data/set1_lund_door/features/descriptors_{0,1}.npy: real OpenCV SIFT descriptors, 5000x128 float32
    from oracle import oracle

    d0 = np.load(os.path.join(REF, "tests/data/set1_lund_door/features/descriptors_0.npy"))
    d1 = np.load(os.path.join(REF, "tests/data/set1_lund_door/features/descriptors_1.npy"))
    assert d0.dtype == np.float32 and d0.shape == (5000, 128)
    # store as uint8 (values are integers in [0,255]); full arrays, 640 KB each
    assert np.array_equal(d0, np.round(d0)) and d0.max() <= 255
    np.savez_compressed(os.path.join(HERE, "lund_door_descriptors.npz"), d0=d0.astype(np.uint8),
                        d1=d1.astype(np.uint8))
    m_full_ratio = oracle.twoway_match(d0, d1, 0.8)
    m_full_noratio = oracle.twoway_match(d0, d1, None)
    m_sub = oracle.twoway_match(d0[:1500], d1[:1500], 0.8)
    np.savez_compressed(os.path.join(HERE, "lund_door_matches_oracle.npz"), full_ratio_0_8=m_full_ratio,
                        full_no_ratio=m_full_noratio, sub1500_ratio_0_8=m_sub)
    print("lund matches: ratio", len(m_full_ratio), "no ratio", len(m_full_noratio), "sub", len(m_sub))


def argoverse_known_answer():
    """tests/frontend/verifier/test_verifier_argoverse.py:41-104: 20 hand-labelled correspondences + intrinsics and
    the expected relative pose. The .pkl is decoded by walking its opcodes with pickletools.genops (nothing in the
    file is executed or imported): it is a dict of four lists of numpy float64 scalars, each carried as 8 raw
    little-endian bytes."""
    import pickletools
    import struct

    path = os.path.join(REF, "tests/data/argoverse/labeled_correspondences/"
                             "argoverse_315975640448534784__315975643412234000.pkl")
    data = open(path, "rb").read()
    vals, cur = {}, None
    for op, arg, _ in pickletools.genops(data):
        if op.name == "SHORT_BINUNICODE" and arg in ("x1", "y1", "x2", "y2"):
            cur = arg
            vals[cur] = []
        elif op.name == "SHORT_BINBYTES" and len(arg) == 8 and cur is not None:
            vals[cur].append(struct.unpack("<d", arg)[0])
    assert all(len(vals[k]) == 20 for k in ("x1", "y1", "x2", "y2"))
    out = dict(vals)
    out.update({
        "fx": 1392.1069298937407, "px": 980.1759848618066, "py": 604.3534182680304,
        "estimation_threshold_px": 0.5,
        "expected_euler_zyx_deg_i1Ri2": [-0.37, 32.47, -0.42], "euler_tol_deg": 1.0,
        "expected_i1ti2": [0.21, -0.0024, 0.976], "translation_tol": 0.01,
        "source": "tests/frontend/verifier/test_verifier_argoverse.py + tests/data/argoverse/labeled_correspondences",
    })
    with open(os.path.join(HERE, "argoverse_known_answer.json"), "w") as f:
        json.dump(out, f, indent=1)


def sampson_known_answers():
    """tests/utils/test_verification_utils.py:49-111 (Sampson / SED closed-form and real-world values)."""
    F_real = [[7.41572822e-09, 4.26005557e-07, -2.61114657e-04], [-4.92270651e-07, 4.29568438e-09, 6.95083578e-04],
              [2.89444929e-04, -1.49345006e-05, -4.01395060e-01]]
    out = {
        "cases": [
            {"F": [[0, 1, 1], [1, 0, 0], [1, 0, 0]], "x1": [[1.0, 3.5], [-2.0, 2.0]], "x2": [[2.0, -1.0], [1.0, 0.0]],
             "sampson": [81 / (21.25 + 4.0), 1 / (13.0 + 2.0)]},
            {"F": F_real, "x1": [[1553, 622], [1553, 622]], "x2": [[357, 662], [818, 517]],
             "sampson": [6.744895e-01, 2.397196e03]},
        ],
        "rtol": 1e-3,
        "source": "tests/utils/test_verification_utils.py:70-111",
    }
    with open(os.path.join(HERE, "sampson_known_answers.json"), "w") as f:
        json.dump(out, f, indent=1)


def lund_door_sift_fixture():
    """DSC_0001.JPG of set1_lund_door as u8 gray (cv.cvtColor RGB2GRAY fixed point, applied by the oracle) and the
    reference's OpenCV SIFT fixture for it (tests/data/set1_lund_door/features/keypoints_0.pkl: coordinates, scales,
    responses of 5000 keypoints; descriptors_0.npy). The .pkl is decoded by walking its opcodes (pickletools.genops):
    the three arrays are the three raw BINBYTES blobs (little-endian float64); nothing in the file is executed."""
    import pickletools

    from PIL import Image

    from oracle import oracle

    data = open(os.path.join(REF, "tests/data/set1_lund_door/features/keypoints_0.pkl"), "rb").read()
    blobs = [arg for op, arg, _ in pickletools.genops(data) if op.name in ("BINBYTES", "BINBYTES8")]
    xy = np.frombuffer(blobs[0], "<f8").reshape(-1, 2)
    scales = np.frombuffer(blobs[1], "<f8")
    responses = np.frombuffer(blobs[2], "<f8")
    assert xy.shape == (5000, 2) and scales.shape == (5000,) and responses.shape == (5000,)
    rgb = np.asarray(Image.open(os.path.join(REF, "tests/data/set1_lund_door/images/DSC_0001.JPG")).convert("RGB"))
    gray = oracle.rgb_to_gray(rgb)
    Image.fromarray(gray).save(os.path.join(HERE, "lund_door_DSC_0001_gray.png"), optimize=True)
    np.savez_compressed(os.path.join(HERE, "lund_door_sift_fixture_0.npz"), xy=xy, scales=scales,
                        responses=responses)


if __name__ == "__main__":
    twoway_known_answers()
    lund_door_descriptors()
    argoverse_known_answer()
    sampson_known_answers()
    lund_door_sift_fixture()

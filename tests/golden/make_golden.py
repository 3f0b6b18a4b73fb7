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


if __name__ == "__main__":
    twoway_known_answers()
    lund_door_descriptors()

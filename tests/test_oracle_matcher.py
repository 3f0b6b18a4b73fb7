"""The matcher oracle (oracle/twoway.c) pinned against the reference's own known answers and fixtures.

Known answers: tests/frontend/matcher/test_twoway_with{,out}ratiotest_matcher.py (reference), committed as data in
tests/golden/twoway_known_answers.json. The Lund-door fixture (real OpenCV SIFT descriptors) gives 3015 ratio-test
matches, as SURVEY.md's independent numpy probe found.
"""
import json
import os

import numpy as np


def test_known_answer_with_ratio(oracle_mod, golden_dir):
    ka = json.load(open(os.path.join(golden_dir, "twoway_known_answers.json")))
    d1 = np.array(ka["descriptors_i1"], np.float32).reshape(-1, 1)
    d2 = np.array(ka["descriptors_i2"], np.float32).reshape(-1, 1)
    np.testing.assert_array_equal(oracle_mod.twoway_match(d1, d2, 0.8), np.array(ka["expected_ratio_0.8"]))


def test_known_answer_without_ratio(oracle_mod, golden_dir):
    ka = json.load(open(os.path.join(golden_dir, "twoway_known_answers.json")))
    d1 = np.array(ka["descriptors_i1"], np.float32).reshape(-1, 1)
    d2 = np.array(ka["descriptors_i2"], np.float32).reshape(-1, 1)
    np.testing.assert_array_equal(oracle_mod.twoway_match(d1, d2, None), np.array(ka["expected_no_ratio"]))


def test_lund_door_subset_matches_golden(oracle_mod, golden_dir):
    z = np.load(os.path.join(golden_dir, "lund_door_descriptors.npz"))
    g = np.load(os.path.join(golden_dir, "lund_door_matches_oracle.npz"))
    d0 = z["d0"].astype(np.float32)
    d1 = z["d1"].astype(np.float32)
    m = oracle_mod.twoway_match(d0[:1500], d1[:1500], 0.8)
    np.testing.assert_array_equal(m, g["sub1500_ratio_0_8"])
    assert len(g["full_ratio_0_8"]) == 3015


def test_output_is_one_to_one_and_sorted(oracle_mod):
    rng = np.random.default_rng(3)
    a = rng.integers(0, 64, size=(300, 16)).astype(np.float32)
    b = np.concatenate([a[:100] + rng.integers(-2, 3, size=(100, 16)), rng.integers(0, 64, size=(200, 16))])
    b = np.clip(b, 0, None).astype(np.float32)
    m = oracle_mod.twoway_match(a, b, 0.8)
    assert len(np.unique(m[:, 0])) == len(m) and len(np.unique(m[:, 1])) == len(m)
    d = np.sqrt(((a[m[:, 0]] - b[m[:, 1]]) ** 2).sum(1))
    assert np.all(np.diff(d) >= 0)


def test_empty_inputs(oracle_mod):
    assert oracle_mod.twoway_match(np.zeros((0, 4), np.float32), np.ones((3, 4), np.float32), 0.8).shape == (0, 2)

"""Squared Sampson distance against the reference's known answers (tests/utils/test_verification_utils.py:86-111,
committed as tests/golden/sampson_known_answers.json), rtol 1e-3 as there:

- the host restatement used by the two-view report's GT metrics (gtsfm_amd/utils/metrics.py);
- the oracle (oracle/ransac.c): its float64 form, and the float32 FMA expression its RANSAC thresholds;
- on the GPU, gtsfm_sampson_sq_batched in both arithmetics: float64 within rtol 1e-3 of the known answers, and the
  verifier's float32 expression bit-identical to the oracle's (the expression the essential-matrix score kernel
  thresholds). The verifier works on K-normalised coordinates, so the pixel-space answer is also checked after
  normalising x by 1000 (F scaled accordingly, distances by 1e-6), the regime the fp32 expression runs in.
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _cases():
    d = json.load(open(os.path.join(HERE, "golden", "sampson_known_answers.json")))
    out = []
    for c in d["cases"]:
        F, x1, x2, exp = (np.array(c[k], np.float64) for k in ("F", "x1", "x2", "sampson"))
        out.append((F, x1, x2, exp))
        S = np.diag([1000.0, 1000.0, 1.0])  # x' = x / 1000  =>  F' = S F S, d' = d / 1e6
        out.append((S @ F @ S, x1 / 1000.0, x2 / 1000.0, exp / 1e6))
    return d["rtol"], out


def test_host_restatement_known_answers():
    from gtsfm_amd.utils import metrics

    rtol, cases = _cases()
    for F, x1, x2, exp in cases:
        np.testing.assert_allclose(metrics.compute_epipolar_distances_sq_sampson(x1, x2, F), exp, rtol=rtol)


def test_oracle_known_answers(oracle_mod):
    rtol, cases = _cases()
    for k, (F, x1, x2, exp) in enumerate(cases):
        np.testing.assert_allclose(oracle_mod.sampson_sq(F, x1, x2, 0), exp, rtol=rtol)
        if k % 2 == 1 or k == 0:  # the float32 verifier expression, in its normalised-coordinate regime
            np.testing.assert_allclose(oracle_mod.sampson_sq(F, x1, x2, 1), exp, rtol=rtol)


@pytest.mark.gpu
def test_gpu_known_answers_and_verifier_arithmetic(oracle_mod):
    import torch

    from gtsfm_amd import device, native

    native.require_gpu()
    rtol, cases = _cases()
    F = torch.tensor(np.stack([c[0] for c in cases]), dtype=torch.float64, device="cuda")
    rows = np.concatenate([np.full(len(c[1]), k) for k, c in enumerate(cases)]).astype(np.int32)
    x1 = np.concatenate([c[1] for c in cases])
    x2 = np.concatenate([c[2] for c in cases])
    exp = np.concatenate([c[3] for c in cases])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    d64 = device.sampson_sq(F, t(rows), t(x1), t(x2), native.GTSFM_SAMPSON_F64).cpu().numpy()
    np.testing.assert_allclose(d64, exp, rtol=rtol)
    d32 = device.sampson_sq(F, t(rows), t(x1), t(x2), native.GTSFM_SAMPSON_F32_VERIFIER).cpu().numpy()
    o32 = np.concatenate([oracle_mod.sampson_sq(c[0], c[1], c[2], 1) for c in cases])
    np.testing.assert_array_equal(d32, o32)
    norm = np.concatenate([np.full(len(c[1]), k % 2 == 1 or k == 0) for k, c in enumerate(cases)])
    np.testing.assert_allclose(d32[norm], exp[norm], rtol=rtol)

"""NetVLADGlobalDescriptor's checkpoint parser against a MATLAB file laid out like the reference's
VGG16-NetVLAD-Pitts30K_struct.mat (netvlad.py:112-152: mat["net"].layers[i].weights, layers 30 / 33,
meta.normalization.averageImage), written here with scipy.io.savemat (the real checkpoint is a download; absent
offline). Checks the mapping the reference applies: conv weights S x S x IN x OUT -> OUT x IN x S x S, score weights
D x K -> K x D x 1, centres negated, whitening 1 x 1 x IN x OUT -> OUT x IN, and the packed blob's layout."""
import numpy as np
import scipy.io

from gtsfm_amd.frontend.global_descriptor.netvlad_global_descriptor import (VGG16_CHANNELS, VGG16_CONV_INDICES,
                                                                             load_netvlad_mat, pack_netvlad_weights)


def test_mat_checkpoint_mapping(tmp_path):
    rng = np.random.default_rng(3)
    layers = np.empty(34, dtype=object)
    for i in range(34):
        layers[i] = {"type": "relu", "weights": np.empty(0, dtype=object)}
    conv = {}
    for idx, (cin, cout) in zip(VGG16_CONV_INDICES, VGG16_CHANNELS):
        cin_s, cout_s = min(cin, 4), min(cout, 5)  # small stand-ins: the parser does not check shapes
        w = rng.standard_normal((3, 3, cin_s, cout_s)).astype(np.float32)
        b = rng.standard_normal(cout_s).astype(np.float32)
        conv[idx] = (w, b)
        wts = np.empty(2, dtype=object)
        wts[0], wts[1] = w, b
        layers[idx] = {"type": "conv", "weights": wts}
    score, cent = rng.standard_normal((6, 3)).astype(np.float32), rng.standard_normal((6, 3)).astype(np.float32)
    white_w, white_b = rng.standard_normal((1, 1, 6, 4)).astype(np.float32), rng.standard_normal(4).astype(np.float32)
    for i, (a, b) in ((30, (score, cent)), (33, (white_w, white_b))):
        wts = np.empty(2, dtype=object)
        wts[0], wts[1] = a, b
        layers[i] = {"type": "x", "weights": wts}
    mean = np.array([[[122.5, 116.0, 103.25]]], np.float32)
    path = tmp_path / "ckpt.mat"
    scipy.io.savemat(str(path), {"net": {"layers": layers, "meta": {"normalization": {"averageImage": mean}}}})
    sd = load_netvlad_mat(path)
    for idx, (w, b) in conv.items():
        np.testing.assert_array_equal(sd[f"backbone.{idx}.weight"], w.transpose(3, 2, 0, 1))
        np.testing.assert_array_equal(sd[f"backbone.{idx}.bias"], b)
    np.testing.assert_array_equal(sd["netvlad.score_proj.weight"], score.T[:, :, None])
    np.testing.assert_array_equal(sd["netvlad.centers"], -cent)
    np.testing.assert_array_equal(sd["whiten.weight"], white_w[0, 0].T)
    np.testing.assert_array_equal(sd["whiten.bias"], white_b)
    np.testing.assert_array_equal(sd["preprocess_mean"], mean.reshape(3))


def test_packed_blob_layout():
    """Full-size random state dict -> blob: offsets as include/gtsfm_hip.h documents (mean[4], per conv W[9][cin][cout]
    + b, score[64][512], centres[512][64], whitening W[4096][32768], b[4096])."""
    import sys
    import os

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    from netvlad_weights import netvlad_state_dict

    sd = netvlad_state_dict(1)
    blob = pack_netvlad_weights(sd)
    np.testing.assert_array_equal(blob[:3], sd["preprocess_mean"])
    o = 4
    for idx, (cin, cout) in zip(VGG16_CONV_INDICES, VGG16_CHANNELS):
        w = sd[f"backbone.{idx}.weight"]
        blk = blob[o: o + 9 * cin * cout].reshape(9, cin, cout)
        assert blk[3 * 1 + 2, 0, cout - 1] == w[cout - 1, 0, 1, 2]
        o += 9 * cin * cout
        np.testing.assert_array_equal(blob[o: o + cout], sd[f"backbone.{idx}.bias"])
        o += cout
    np.testing.assert_array_equal(blob[o: o + 64 * 512], sd["netvlad.score_proj.weight"].reshape(-1))
    o += 64 * 512
    np.testing.assert_array_equal(blob[o: o + 512 * 64], sd["netvlad.centers"].reshape(-1))
    o += 512 * 64
    assert blob[o + 4096 * 32768 - 1] == sd["whiten.weight"][-1, -1]
    o += 4096 * 32768
    np.testing.assert_array_equal(blob[o:], sd["whiten.bias"])

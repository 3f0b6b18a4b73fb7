"""Diagnostic: per-wave cycle split (M, barrier, E, barrier) of the four-waves-per-SIMD distance GEMM (GTSFM_MNN=q5)
over one grouped 100-image launch. Usage: GTSFM_MNN=q5 python tools/qstamps.py"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gtsfm_amd import device, native  # noqa: E402

n_img, K = 100, 2048
rng = np.random.default_rng(3)
x = rng.gamma(0.6, 1.0, size=(n_img, K, 128)).astype(np.float32)
x = np.clip(np.round(x / np.linalg.norm(x, axis=2, keepdims=True) * 512), 0, 255).astype(np.float32)
dev = torch.device("cuda")
desc = torch.from_numpy(x).to(dev)
counts = torch.full((n_img,), K, dtype=torch.int32, device=dev)
pairs_np = np.array([(i, j) for i in range(n_img) for j in range(i + 1, n_img)], np.int32)
pairs = torch.from_numpy(pairs_np).to(dev)
G = device.match_group_size(K, 128)
groups = torch.from_numpy(device.pair_groups(pairs_np, G)).to(dev)
L = native.lib()
buf = (ctypes.c_ulonglong * 128)()
device.match_pairs(desc, counts, pairs, 0.8, groups=groups)
L.gtsfm_diag_mnn_q_stamps(buf)
device.match_pairs(desc, counts, pairs, 0.8, groups=groups)
L.gtsfm_diag_mnn_q_stamps(buf)
units = len(pairs_np) * 4 * 32
ncol = 8 if os.environ.get("GTSFM_MNN") == "rs" else 6
st = np.array(list(buf), np.float64).reshape(16, 8)[:, :ncol] / units
print(json.dumps({"cycles_per_unit_per_wave": st.round(0).tolist(),
                  "mean_by_role": [st[4 * r: 4 * r + 4].mean(0).round(0).tolist() for r in range(4)]}))

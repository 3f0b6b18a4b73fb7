"""Distance-GEMM microbench: all pairs of N synthetic SIFT-like images at 2048 keypoints, whole match_pairs call and the
mnn kernel alone (HIP events through gtsfm_match_set_kernel_events), without and with block-tiled pair groups.
Usage: python tools/matchbench.py [N]"""
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gtsfm_amd import device, native  # noqa: E402

n_img = int(sys.argv[1]) if len(sys.argv) > 1 else 100
K = 2048
rng = np.random.default_rng(3)
x = rng.gamma(0.6, 1.0, size=(n_img, K, 128)).astype(np.float32)
x = np.clip(np.round(x / np.linalg.norm(x, axis=2, keepdims=True) * 512), 0, 255).astype(np.float32)
n_pl = int(0.3 * K)  # planted: 30% of the keypoints share a latent descriptor (+ integer noise) across images
x[:, :n_pl] = np.clip(x[0, :n_pl][None] + rng.integers(-8, 9, size=(n_img, n_pl, 128)), 0, 255)
dev = torch.device("cuda")
desc = torch.from_numpy(x).to(dev)
counts = torch.full((n_img,), K, dtype=torch.int32, device=dev)
pairs_np = np.array([(i, j) for i in range(n_img) for j in range(i + 1, n_img)], np.int32)
pairs = torch.from_numpy(pairs_np).to(dev)
P = len(pairs_np)
flops = 2.0 * K * K * 128 * P
L = native.lib()
G = device.match_group_size(K, 128)
out = {"pairs": P, "group_size": G}
for name, groups in (("ungrouped", None), ("grouped", torch.from_numpy(device.pair_groups(pairs_np, G)).to(dev))):
    for _ in range(2):
        device.match_pairs(desc, counts, pairs, 0.8, groups=groups)
    torch.cuda.synchronize()
    t = time.time()
    reps = 5
    for _ in range(reps):
        idx, cnt = device.match_pairs(desc, counts, pairs, 0.8, groups=groups)
    torch.cuda.synchronize()
    dt = (time.time() - t) / reps
    kev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for e in kev:
        e.record()
    kms = []
    native.check(L.gtsfm_match_set_kernel_events(kev[0].cuda_event, kev[1].cuda_event), "events")
    for _ in range(3):
        device.match_pairs(desc, counts, pairs, 0.8, groups=groups)
        torch.cuda.synchronize()
        kms.append(kev[0].elapsed_time(kev[1]))
    native.check(L.gtsfm_match_set_kernel_events(None, None), "events")
    km = float(np.median(kms))
    out[name] = {"call_ms": round(dt * 1e3, 3), "kernel_ms": round(km, 3),
                 "kernel_TFLOPs": round(flops / (km * 1e-3) / 1e12, 1),
                 "kernel_frac_f16_peak": round(flops / (km * 1e-3) / 2.5e15, 4),
                 "mean_matches": float(cnt.float().mean()),
                 "checksum": hashlib.sha1(cnt.cpu().numpy().tobytes() + idx.cpu().numpy().tobytes()).hexdigest()[:16]}
print(json.dumps(out))
if hasattr(L, "gtsfm_pp_stamps"):  # diagnostic build: per-wave cycles of one grouped launch
    import ctypes
    buf = (ctypes.c_ulonglong * 64)()
    L.gtsfm_pp_stamps(buf)  # clear
    device.match_pairs(desc, counts, pairs, 0.8, groups=torch.from_numpy(device.pair_groups(pairs_np, G)).to(dev))
    L.gtsfm_pp_stamps(buf)
    units = P * 4 * 32  # 2048 rows: 4 passes x 32 column units per pair
    st = np.array(list(buf), np.float64).reshape(8, 8) / units
    print(json.dumps({"cycles_per_unit_per_wave [M, bar1, E, bar2, E.rows, E.colkeys, E.atomics, E.rest]":
                      st.round(0).tolist()}))

"""Temporary matcher-stage microbench (superseded by bench.py)."""
import sys, time, json
import numpy as np, torch
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gtsfm_amd import device, native
n_img = int(sys.argv[1]) if len(sys.argv) > 1 else 100
K = 2048
rng = np.random.default_rng(3)
x = rng.gamma(0.6, 1.0, size=(n_img, K, 128)).astype(np.float32)
x = np.clip(np.round(x / np.linalg.norm(x, axis=2, keepdims=True) * 512), 0, 255).astype(np.float32)
dev = torch.device('cuda')
desc = torch.from_numpy(x).to(dev)
counts = torch.full((n_img,), K, dtype=torch.int32, device=dev)
pairs = torch.tensor([(i, j) for i in range(n_img) for j in range(i + 1, n_img)], dtype=torch.int32, device=dev)
for _ in range(2):
    device.match_pairs(desc, counts, pairs, 0.8)
torch.cuda.synchronize()
t = time.time(); reps = 5
for _ in range(reps):
    idx, cnt = device.match_pairs(desc, counts, pairs, 0.8)
torch.cuda.synchronize()
dt = (time.time() - t) / reps
P = pairs.shape[0]
flops = 2.0 * K * K * 128 * P
print(json.dumps({"pairs": P, "ms": dt * 1e3, "pairs_per_s": P / dt, "TFLOPs": flops / dt / 1e12,
                  "mean_matches": float(cnt.float().mean())}))

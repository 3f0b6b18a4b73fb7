"""C3 end to end probe: HIP SuperPoint (seeded random weights) on n rendered 1080p images at 4096 keypoints, then all
pairs through GTSFM_MATCH_F16_RERANK (ratio 0.8); times extraction and matching and checks a sample of pairs against
EXACT_F32. Usage: python tools/sp_matchbench.py [n_images]"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from gtsfm_amd import device, native, synthetic  # noqa: E402
from gtsfm_amd.frontend.detector_descriptor.superpoint import pack_superpoint_weights  # noqa: E402
from superpoint_weights import superpoint_state_dict  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
dev = torch.device("cuda")
native.lib()
scene = synthetic.render_scene(n, 1080, 1920, device="cuda")
w = torch.from_numpy(pack_superpoint_weights(superpoint_state_dict(0))).to(dev)
res = device.superpoint_extract(scene.images, w, 4096)
torch.cuda.synchronize()
t = time.perf_counter()
res = device.superpoint_extract(scene.images, w, 4096)
torch.cuda.synchronize()
t_sp = time.perf_counter() - t
desc, cnt = res.desc.contiguous(), res.count.contiguous()
pairs = torch.tensor([(i, j) for i in range(n) for j in range(i + 1, n)], dtype=torch.int32, device=dev)
P = pairs.shape[0]
device.match_pairs(desc, cnt, pairs, 0.8, native.GTSFM_MATCH_F16_RERANK)
torch.cuda.synchronize()
t = time.perf_counter()
idx, m = device.match_pairs(desc, cnt, pairs, 0.8, native.GTSFM_MATCH_F16_RERANK)
torch.cuda.synchronize()
t_m = time.perf_counter() - t
sub = pairs[: min(P, 6)].contiguous()
ie, me = device.match_pairs(desc, cnt, sub, 0.8, native.GTSFM_MATCH_EXACT_F32)
same = all(torch.equal(ie[p, : me[p]], idx[p, : m[p]]) and int(me[p]) == int(m[p]) for p in range(sub.shape[0]))
print(json.dumps({"images": n, "pairs": P, "kpts_mean": float(cnt.float().mean()), "superpoint_ms_per_image":
                  round(t_sp / n * 1e3, 3), "match_ms_per_pair": round(t_m / P * 1e3, 3),
                  "mean_matches": float(m.float().mean()), "sample_identical_to_exact": same}), flush=True)

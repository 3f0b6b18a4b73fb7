"""Concurrency probe: SIFT extraction of the C2 images and the C2 RANSAC verification, each alone and both at once on
two streams (HIP events around each). Tells how much of verify a cross-step pipeline could hide under extraction.

    python tools/overlap_probe.py [n_images]
"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from gtsfm_amd import device, synthetic  # noqa: E402
from gtsfm_amd.frontend.all_pairs import AllPairsFrontEnd, FrontEndConfig  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dev = torch.device("cuda")
scene = synthetic.render_scene(n, 1080, 1920, device="cuda")
host = scene.images.cpu().pin_memory()
fe = AllPairsFrontEnd(host, scene.intrinsics, n, 0, 1, dev, FrontEndConfig())
fe.step(resident=False)
fe.step(resident=True)
torch.cuda.synchronize()
idx, cnt = fe.d_match[0][: fe.P], fe.d_match[1][: fe.P]
xy = fe.feats.xy.clone()
s_ex, s_ver = torch.cuda.Stream(), torch.cuda.Stream()


def extract():
    fe._extract(resident=True)


def verify():
    device.ransac_essential(xy, fe.intr, fe.pairs_dev, idx, cnt, 4.0, pair_id_base=0)


def timed(fn, stream, reps=5):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        ev[0].record()
        for _ in range(reps):
            fn()
        ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


for _ in range(2):
    timed(extract, s_ex, 1)
    timed(verify, s_ver, 1)
t_ex = timed(extract, s_ex)
t_ver = timed(verify, s_ver)
reps = 5
torch.cuda.synchronize()
t0 = time.perf_counter()
with torch.cuda.stream(s_ex):
    for _ in range(reps):
        extract()
with torch.cuda.stream(s_ver):
    for _ in range(reps):
        verify()
torch.cuda.synchronize()
t_both = (time.perf_counter() - t0) * 1e3 / reps
print(f"extract alone {t_ex:.2f} ms, verify alone {t_ver:.2f} ms, sum {t_ex + t_ver:.2f} ms; "
      f"both on two streams {t_both:.2f} ms per (extract + verify) -> hidden {t_ex + t_ver - t_both:.2f} ms")

"""C3-shaped float matching microbench: n images x 4096 SuperPoint-like 256-D unit descriptors (30% planted matches),
all pairs through GTSFM_MATCH_F16_RERANK (and a sample through EXACT_F32); reports ms/pair and the shortlist GEMM's
fp16 MFMA rate (2 sides x 2*K1*K2*D flop per pair)."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from gtsfm_amd import device, native  # noqa: E402

n, K, D = int(sys.argv[1]) if len(sys.argv) > 1 else 40, 4096, 256
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(3)
latent = torch.nn.functional.normalize(torch.randn(K, D, device=dev, generator=g), dim=1)
desc = torch.nn.functional.normalize(torch.randn(n, K, D, device=dev, generator=g), dim=2)
k = int(0.3 * K)
for i in range(n):
    rows = torch.randperm(K, device=dev, generator=g)[:k]
    src = torch.randperm(K, device=dev, generator=g)[:k]
    desc[i, rows] = torch.nn.functional.normalize(latent[src] + 0.15 / 16 * torch.randn(k, D, device=dev, generator=g),
                                                  dim=1)
desc = desc.contiguous()
cnt = torch.full((n,), K, dtype=torch.int32, device=dev)
pairs = torch.tensor([(i, j) for i in range(n) for j in range(i + 1, n)], dtype=torch.int32, device=dev)
P = pairs.shape[0]
L = native.lib()


def run(mode, pr):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for e in ev:
        e.record()
    L.gtsfm_match_set_kernel_events(ev[0].cuda_event, ev[1].cuda_event)
    torch.cuda.synchronize()
    t = time.perf_counter()
    idx, m = device.match_pairs(desc, cnt, pr, 0.8, mode)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) * 1e3
    L.gtsfm_match_set_kernel_events(None, None)
    return idx, m, wall, ev[0].elapsed_time(ev[1])


run(native.GTSFM_MATCH_F16_RERANK, pairs)
idx, m, wall, kms = run(native.GTSFM_MATCH_F16_RERANK, pairs)
flop = 2 * 2.0 * K * K * D * P
print(f"F16_RERANK: {P} pairs, {wall:.1f} ms ({wall / P:.3f} ms/pair, {P / wall * 1e3:.0f} pairs/s); shortlist kernel "
      f"{kms:.2f} ms = {flop / kms / 1e9:.0f} TFLOP/s fp16; mean matches {m.float().mean().item():.0f}", flush=True)
sub = pairs[: min(P, 24)].contiguous()
ie, me, we, _ = run(native.GTSFM_MATCH_EXACT_F32, sub)
ir, mr, wr, _ = run(native.GTSFM_MATCH_F16_RERANK, sub)
same = torch.equal(me, mr) and all(torch.equal(ie[p, : me[p]], ir[p, : mr[p]]) for p in range(sub.shape[0]))
print(f"EXACT_F32: {sub.shape[0]} pairs {we:.1f} ms ({we / sub.shape[0]:.2f} ms/pair); identical to F16_RERANK: {same}")

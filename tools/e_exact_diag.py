"""Pair-by-pair E / R / t differences between the HIP verifier and the oracle on tests/test_verifier_gpu.py's batched
scene, and the five-point candidates of the first launch (read from the workspace's candidate buffer) against
oracle_sample5 + oracle_five_point (development diagnostic for the bit-exact E path)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gtsfm_amd import device  # noqa: E402
from oracle import oracle as oracle_mod  # noqa: E402
from tests import scenes  # noqa: E402


def main():
    rng = np.random.default_rng(12)
    n_pairs = 40
    kps, Ks, Ms = [], [], []
    for p in range(n_pairs):
        n_in = int(rng.integers(10, 700))
        n_out = int(n_in * rng.uniform(0.4, 1.5)) if p % 7 else 0
        kp1, kp2, K, R, t, inl = scenes.random_two_view(rng, n_in, n_out)
        kps.append((kp1, kp2))
        Ks.append(K)
        Ms.append(len(kp1))
    kmax = max(Ms)
    kp = np.zeros((2 * n_pairs, kmax, 2), np.float32)
    intr = np.zeros((2 * n_pairs, 3))
    pairs = np.zeros((n_pairs, 2), np.int32)
    mi = np.zeros((n_pairs, kmax, 2), np.int32)
    for p, ((a, b), K) in enumerate(zip(kps, Ks)):
        kp[2 * p, : len(a)] = a
        kp[2 * p + 1, : len(b)] = b
        intr[2 * p] = intr[2 * p + 1] = (K[0, 0], K[0, 2], K[1, 2])
        pairs[p] = (2 * p, 2 * p + 1)
        mi[p, : Ms[p]] = np.arange(Ms[p])[:, None]
    dev = torch.device("cuda")
    from gtsfm_amd import native

    L = native.lib()
    P, mcap = n_pairs, kmax
    wsb = L.gtsfm_ransac_workspace_bytes(P, mcap)
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    E = torch.zeros((P, 3, 3), dtype=torch.float64, device=dev)
    R = torch.zeros_like(E)
    t = torch.zeros((P, 3), dtype=torch.float64, device=dev)
    n_inl = torch.zeros((P,), dtype=torch.int32, device=dev)
    status, n_hyp, n_models = torch.zeros_like(n_inl), torch.zeros_like(n_inl), torch.zeros_like(n_inl)
    mask = torch.zeros((P, mcap), dtype=torch.uint8, device=dev)
    ptr = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    tk = [torch.from_numpy(a).to(dev) for a in (kp, intr, pairs, mi)]
    cnt = torch.tensor(Ms, dtype=torch.int32, device=dev)
    rc = L.gtsfm_ransac_E_batched(ptr(tk[0]), ptr(tk[1]), 2 * P, kmax, ptr(tk[2]), P, ptr(tk[3]), ptr(cnt), mcap, 4.0,
                                  0.999999, 1000, native.GTSFM_RANSAC_SCORING_MSAC, native.RANSAC_DEFAULT_SEED, 0, None,
                                  ptr(ws), wsb, ptr(E), ptr(R), ptr(t), ptr(n_inl), ptr(status), ptr(n_hyp),
                                  ptr(n_models), ptr(mask), None)
    native.check(rc, "gtsfm_ransac_E_batched")
    torch.cuda.synchronize()
    E, R, t = E.cpu().numpy(), R.cpu().numpy(), t.cpu().numpy()
    nh = n_hyp.cpu().numpy()
    # workspace layout (ransac.hip ransac_layout): x1n, x2n, pts, PairState, cand [P][10][9][512], nsol [P][512]
    al = lambda n: (n + 255) // 256 * 256  # noqa: E731
    o = 2 * al(P * mcap * 16) + al(P * mcap * 16) + al(P * 112)
    raw = ws.cpu().numpy()
    cand = raw[o: o + P * 10 * 9 * 512 * 8].view(np.float64).reshape(P, 10, 9, 512)
    o += al(P * 512 * 10 * 9 * 8)
    nsol = raw[o: o + P * 512 * 4].view(np.int32).reshape(P, 512)
    o += al(P * 512 * 4)
    stage = raw[o: o + P * 96 * 512 * 8].view(np.float64).reshape(P, 96, 512)
    hip_N, hip_R = [], []
    og = None
    og_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "abvar", "libog.so")
    if os.path.exists(og_path):  # the oracle's five-point compiled for the GPU (tools/ubench/og_build.sh)
        og = ctypes.CDLL(og_path)
        og.og_five_point_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 4
    samples, cpu_E, hip_E = [], [], []
    n_cmp = n_diff = n_cnt = 0
    worst = 0.0
    diffs = []
    for p in range(P):
        if nh[p] > 64:
            continue  # later launches reuse the buffer: only single-chunk pairs keep chunk 0's candidates
        K = Ks[p]
        a, b = kps[p]
        x1 = (a.astype(np.float32).astype(np.float64) - K[:2, 2]) / K[0, 0]
        x2 = (b.astype(np.float32).astype(np.float64) - K[:2, 2]) / K[0, 0]
        for h in range(64):
            idx = oracle_mod.sample5(p, h, Ms[p], native.RANSAC_DEFAULT_SEED)
            Es = oracle_mod.five_point(x1[idx], x2[idx]) if idx is not None else np.zeros((0, 3, 3))
            if len(Es) != nsol[p, h]:
                n_cnt += 1
                continue
            if idx is not None:
                samples.append((x1[idx], x2[idx]))
                cpu_E.append(Es)
                hip_E.append(cand[p, : len(Es), :, h].copy())
                hip_R.append(stage[p, :60, h].copy())
                hip_N.append(stage[p, 60:96, h].copy())
            for s_ in range(len(Es)):
                g = cand[p, s_, :, h]
                d = np.abs(g - Es[s_].reshape(9)).max()
                n_cmp += 1
                n_diff += d > 0
                worst = max(worst, d)
                diffs.append(d)
    diffs = np.array(diffs)
    print(f"five-point candidates (HIP solver vs CPU oracle): {n_cmp} compared, {n_diff} differ (max {worst:.3e}, "
          f"median {np.median(diffs):.3e}), {n_cnt} solution-count mismatches", flush=True)
    if og is not None and samples:
        n = len(samples)
        X1 = np.ascontiguousarray(np.stack([a for a, _ in samples]), np.float64)
        X2 = np.ascontiguousarray(np.stack([b for _, b in samples]), np.float64)
        gE = np.zeros((n, 90))
        gn = np.zeros(n, np.int32)
        gN = np.zeros((n, 36))
        gR = np.zeros((n, 60))
        og.og_five_point_batch(X1.ctypes.data, X2.ctypes.data, n, gE.ctypes.data, gn.ctypes.data, gN.ctypes.data,
                               gR.ctypes.data)
        dN = np.array([np.abs(gN[i] - hip_N[i]).max() for i in range(n)])
        dR = np.array([np.abs(gR[i] - hip_R[i]).max() for i in range(n)])
        print(f"stage 1 vs the oracle: N differs on {(dN > 0).sum()} of {n} samples (max {dN.max():.3e}); reduced rows "
              f"differ on {(dR > 0).sum()} (max {dR.max():.3e})", flush=True)
        d_cpu = d_hip = cnt_bad = 0
        for i in range(n):
            if gn[i] != len(cpu_E[i]):
                cnt_bad += 1
                continue
            ge = gE[i, : 9 * gn[i]].reshape(-1, 9)
            d_cpu += int((ge != cpu_E[i].reshape(-1, 9)).any())
            d_hip += int((ge != hip_E[i]).any())
        print(f"oracle five-point compiled for the GPU: {n} samples; differs from the CPU oracle on {d_cpu}, from the "
              f"HIP solver on {d_hip}; solution-count mismatches {cnt_bad}", flush=True)
    n_e = n_r = 0
    for p in range(n_pairs):
        K = Ks[p]
        a, b = kps[p]
        x1 = (a.astype(np.float32).astype(np.float64) - K[:2, 2]) / K[0, 0]
        x2 = (b.astype(np.float32).astype(np.float64) - K[:2, 2]) / K[0, 0]
        rE, rmask, rR, rt, rn, rh = oracle_mod.ransac_E(x1, x2, 4.0 / K[0, 0], pair_id=p)
        de = np.abs(E[p].reshape(9) - np.asarray(rE).reshape(9)).max()
        dr = np.abs(R[p] - rR).max()
        n_e += de > 0
        n_r += dr > 0
        print(f"pair {p:2d} M {Ms[p]:5d} inliers {rn:5d}  |dE| {de:.3e}  |dR| {dr:.3e}  |dt| {np.abs(t[p] - rt).max():.3e}")
    print(f"pairs with E differing: {n_e} of {n_pairs}; R differing: {n_r}")


if __name__ == "__main__":
    main()

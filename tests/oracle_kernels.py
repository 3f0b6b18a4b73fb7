"""Test stand-in for gtsfm_amd.frontend.all_pairs.HipKernels: the same kernel-set calls computed by the CPU oracle on CPU
tensors, so AllPairsFrontEnd's host logic (chunking, sharding, all-gather, compaction, D2H assembly) runs under gloo
without a GPU. Test infrastructure only -- never imported by the product package."""
from __future__ import annotations

import numpy as np
import torch

from oracle import oracle


class OracleRansacResult:
    def __init__(self, P, mcap):
        self.R = torch.zeros((P, 3, 3), dtype=torch.float64)
        self.E = torch.zeros((P, 3, 3), dtype=torch.float64)
        self.t = torch.zeros((P, 3), dtype=torch.float64)
        self.n_inliers = torch.zeros(P, dtype=torch.int32)
        self.status = torch.zeros(P, dtype=torch.int32)
        self.n_hyp = torch.zeros(P, dtype=torch.int32)
        self.mask = torch.zeros((P, mcap), dtype=torch.uint8)
        self.n_models = None


class OracleKernels:
    attr_dim, desc_dim = 3, 128
    gather = (("xy", None), ("desc", torch.uint8), ("count", None))
    max_pair_chunk = None

    def extract_workspace_bytes(self, n, H, W, kpts):
        return 0

    def extract(self, images, kpts, out, workspace):
        for i in range(images.shape[0]):
            img = images[i].numpy()
            gray = oracle.rgb_to_gray(img) if img.ndim == 3 else img
            kp, desc, nd = oracle.sift(gray, kpts)
            n = len(kp)
            out.xy[i].zero_()
            out.desc[i].zero_()
            out.xy[i, :n] = torch.from_numpy(kp[:, :2])
            out.attr[i, :n] = torch.from_numpy(kp[:, 2:5])
            out.desc[i, :n] = torch.from_numpy(desc)
            out.count[i] = n
            out.n_detected[i] = nd

    def match(self, f, pairs, ratio, groups=None, image_hw=None):  # groups only lay out GPU work
        desc, counts = f.desc, f.count
        P, kmax = pairs.shape[0], desc.shape[1]
        idx = torch.zeros((P, kmax, 2), dtype=torch.int32)
        cnt = torch.zeros(P, dtype=torch.int32)
        for p in range(P):
            i1, i2 = int(pairs[p, 0]), int(pairs[p, 1])
            m = oracle.twoway_match(desc[i1, : int(counts[i1])].numpy(), desc[i2, : int(counts[i2])].numpy(), ratio)
            m = m.reshape(-1, 2)
            idx[p, : len(m)] = torch.from_numpy(m.astype(np.int64).astype(np.int32))
            cnt[p] = len(m)
        return idx, cnt

    def verify(self, xy, intr, pairs, idx, cnt, thresh_px, pair_ids):
        P, mcap = idx.shape[0], idx.shape[1]
        res = OracleRansacResult(P, mcap)
        for p in range(P):
            i1, i2 = int(pairs[p, 0]), int(pairs[p, 1])
            M = int(cnt[p])
            if M < 6:
                res.status[p] = 1
                continue
            m = idx[p, :M].numpy().astype(np.int64)
            f1, u1, v1 = intr[i1].tolist()
            f2, u2, v2 = intr[i2].tolist()
            x1 = (xy[i1, m[:, 0]].numpy().astype(np.float64) - [u1, v1]) / f1
            x2 = (xy[i2, m[:, 1]].numpy().astype(np.float64) - [u2, v2]) / f2
            r = oracle.ransac_E(x1, x2, thresh_px / max(f1, f2), pair_id=int(pair_ids[p]))
            if r is None:
                res.status[p] = 2
                continue
            E, mask, R, t, n, nh = r
            res.E[p] = torch.from_numpy(E)
            res.R[p] = torch.from_numpy(R)
            res.t[p] = torch.from_numpy(t)
            res.n_inliers[p] = n
            res.n_hyp[p] = nh
            res.mask[p, :M] = torch.from_numpy(mask)
        return res

    def bundle_adjust(self, xy, intr, pairs, idx, cnt, res, min_inliers, max_iters, reproj_thresh, tri_thresh):
        """oracle/ba2.c on every verified pair with >= min_inliers rows (two_view_estimator.py:311-337)."""
        P, mcap = idx.shape[0], idx.shape[1]
        out = OracleRansacResult(P, mcap)
        out.status = res.status.clone()
        for p in range(P):
            M = int(cnt[p])
            rows = np.flatnonzero(res.mask[p, :M].numpy())
            out.R[p], out.t[p] = res.R[p], res.t[p]
            if int(res.status[p]) != 0 or len(rows) < min_inliers:
                out.mask[p] = res.mask[p]
                out.n_inliers[p] = len(rows)
                continue
            i1, i2 = int(pairs[p, 0]), int(pairs[p, 1])
            m = idx[p, rows].numpy().astype(np.int64)
            uv1 = xy[i1, m[:, 0]].numpy().astype(np.float64)
            uv2 = xy[i2, m[:, 1]].numpy().astype(np.float64)
            st, R, t, valid, _, _ = oracle.ba2(uv1, uv2, intr[i1].numpy(), intr[i2].numpy(), res.R[p].numpy(),
                                               res.t[p].numpy(), max_iters, reproj_thresh, tri_thresh)
            out.R[p], out.t[p] = torch.from_numpy(R), torch.from_numpy(t)
            out.mask[p, rows[valid]] = 1
            out.n_inliers[p] = int(valid.sum())
        return out

    def compact(self, idx, cnt, res, min_inliers, min_ratio, capacity, out_offsets, out_v_corr, out_isp_ok,
                ratio_inliers=None):
        """numpy restatement of gtsfm_compact_verified (opencv_verifier_base.py:98-101 +
        inlier_support_processor.py:73-87)."""
        pos = 0
        for p in range(idx.shape[0]):
            out_offsets[p] = pos
            st, n, M = int(res.status[p]), int(res.n_inliers[p]), int(cnt[p])
            nr = n if ratio_inliers is None else int(ratio_inliers[p])
            ratio = nr / M if (st == 0 and M > 0) else 0.0
            out_isp_ok[p] = int(st == 0 and not (ratio < min_ratio or (0 < n < min_inliers)))
            if st != 0:
                continue
            rows = idx[p, :M][res.mask[p, :M].bool()]
            out_v_corr[pos: pos + len(rows)] = rows
            pos += len(rows)
        out_offsets[idx.shape[0]] = pos

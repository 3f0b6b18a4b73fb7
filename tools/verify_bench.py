"""A/B timing of library variants on the C2 front-end (development tool).

Runs AllPairsFrontEnd on the C2 scene (100 rendered 1080p images, 4950 pairs) with the library named by
GTSFM_HIP_LIB (default: the in-tree product build), prints the median per-stage milliseconds of 3 instrumented
device-resident steps as one JSON line, and compares the per-pair verifier results with a reference run saved by the
first invocation (gpurun_out/verify_ref.npz): status, inlier counts, hypothesis counts and R must match, so a
variant that changes results is flagged.

    for v in build_var/libgtsfm_hip_*.so; do GTSFM_HIP_LIB=$v python tools/verify_bench.py; done
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from gtsfm_amd import native, synthetic  # noqa: E402
from gtsfm_amd.frontend.all_pairs import AllPairsFrontEnd, FrontEndConfig  # noqa: E402


def main():
    n = int(os.environ.get("VB_IMAGES", "100"))
    scene = synthetic.render_scene(n, 1080, 1920, device="cuda")
    host = scene.images.cpu().pin_memory()
    del scene.images
    fe = AllPairsFrontEnd(host, scene.intrinsics, n, 0, 1, torch.device("cuda"), FrontEndConfig())
    res = fe.step()
    fe.step(resident=True)
    fe.instrument = True
    rows = []
    for _ in range(3):
        fe.step(resident=True)
        torch.cuda.synchronize()
        rows.append(fe.stage_ms())
    st = {k: round(float(np.median([r[k] for r in rows])), 3) for k in rows[0]}
    n_hyp = fe.stats["n_hyp"].cpu().numpy()
    ref_path = os.path.join(REPO, "gpurun_out", "verify_ref.npz")
    cur = dict(status=res.status, n_inliers=res.n_inliers, n_hyp=n_hyp, R=res.R)
    same = None
    if os.path.exists(ref_path):
        ref = np.load(ref_path)
        same = {k: bool(np.array_equal(ref[k], cur[k])) for k in ("status", "n_inliers", "n_hyp")}
        same["R_maxdiff"] = float(np.abs(ref["R"] - cur["R"]).max())
        same["n_inliers_diff_pairs"] = int((ref["n_inliers"] != cur["n_inliers"]).sum())
    else:
        os.makedirs(os.path.dirname(ref_path), exist_ok=True)
        np.savez(ref_path, **cur)
    print(json.dumps({"lib": os.path.relpath(native.LIB_PATH, REPO), "stage_ms": st,
                      "hyp_total": int(n_hyp.sum()),
                      "hyp_chunks_hist": np.bincount((n_hyp + 63) // 64, minlength=17).tolist(), "same_as_ref": same}), flush=True)


if __name__ == "__main__":
    main()

"""Per-phase shader-clock cycles of the RANSAC kernels over one C2 front-end step (development instrumentation).

Needs the -DGTSFM_RANSAC_PROF build of ransac.hip (tools/build_variants_src.sh gtsfm_amd/csrc/ransac.hip
prof:-DGTSFM_RANSAC_PROF), selected with GTSFM_HIP_LIB=build_var/libgtsfm_hip_prof.so. Cycles are summed over waves
(lane 0 of each wave adds its own phase time), so the table is the phase mix of wave-time, not wall time.

    GTSFM_HIP_LIB=build_var/libgtsfm_hip_prof.so python tools/ransac_prof.py [n_images]
"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from gtsfm_amd import native, synthetic  # noqa: E402
from gtsfm_amd.frontend.all_pairs import AllPairsFrontEnd, FrontEndConfig  # noqa: E402

NAMES = {0: "s1 sample+load", 1: "s1 nullspace", 2: "s1 A rows", 3: "s1 Gauss-Jordan", 4: "s1 store",
         5: "s2 load", 6: "s2 B + det poly", 7: "s2 Sturm chain", 8: "s2 isolation", 9: "s2 bisection",
         10: "s2 Newton", 11: "s2 E from roots + store", 12: "s2 tail", 13: "score: candidates", 14: "score: chunk sync",
         22: "refine: first MSAC", 23: "refine: GC labels (keys+sort+runs)", 24: "refine: refits", 25: "refine: MSAC of refit",
         26: "refine: final mask", 27: "refine: recoverPose"}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    L = native.lib()
    fn = L.gtsfm_ransac_prof_read
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    scene = synthetic.render_scene(n, 1080, 1920, device="cuda")
    host = scene.images.cpu().pin_memory()
    fe = AllPairsFrontEnd(host, scene.intrinsics, n, 0, 1, torch.device("cuda"), FrontEndConfig())
    fe.step(resident=False)
    buf = (ctypes.c_ulonglong * 32)()
    fn(buf, 1)
    fe.step(resident=True)
    fn(buf, 1)
    c = np.array(buf[:], dtype=np.float64)
    tot = {"solve1": c[0:5].sum(), "solve2": c[5:13].sum(), "score": c[13:15].sum(), "refine": c[22:28].sum()}
    print(f"waves: solve1 {int(c[16])}  solve2 {int(c[17])}  score workgroups {int(c[18])}")
    print(f"isolation iterations (lane 0 sum) {int(c[20])}, real roots (lane 0 sum) {int(c[21])}")
    print(f"refine: GC iterations {int(c[28])}, of which bitonic sort cycles {c[29]:.4g} (inside 'GC labels')")
    allt = sum(tot.values())
    for k, name in NAMES.items():
        print(f"{name:26s} {c[k]:14.4g} cycles  {100 * c[k] / allt:5.1f} % of all wave-cycles")
    for k, v in tot.items():
        print(f"{k:10s} {100 * v / allt:5.1f} %")


if __name__ == "__main__":
    main()

"""Phase timing of ransac_solve_kernel (instrumented build in gtsfm_amd/_lib/prof, not the product)."""
import ctypes, os, sys, time
import numpy as np, torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from gtsfm_amd import native
native.LIB_PATH = os.path.join(REPO, "gtsfm_amd", "_lib", "prof", "libgtsfm_hip.so")
from gtsfm_amd import device as hip, synthetic
import bench
L = native.lib()
L.gtsfm_ransac_profile.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
n = 100
scene = synthetic.render_scene(n, 1080, 1920, device="cuda")
fe = bench.FrontEnd(scene.images, scene.intrinsics, n, 2048, 0, 1)
_, (feats, idx, mcnt, res) = fe.step()
torch.cuda.synchronize()
buf0 = (ctypes.c_ulonglong * 16)(); L.gtsfm_ransac_profile(buf0)
t = time.time()
r = hip.ransac_essential(feats.xy, fe.intr, fe.pairs, idx, mcnt, 4.0)
torch.cuda.synchronize(); dt = time.time() - t
buf1 = (ctypes.c_ulonglong * 16)(); L.gtsfm_ransac_profile(buf1)
d = np.array(buf1[:9], dtype=np.float64) - np.array(buf0[:9], dtype=np.float64)
names = ["sample+load", "nullspace", "A det rows", "EEt rows + GJ", "B + det poly", "sturm chain", "isolation",
         "bisection", "E from roots + store"]
tot = d.sum()
print("verify wall ms %.1f; hyps %d" % (dt * 1e3, int(r.n_hyp.sum())))
for k in range(9):
    print("%-22s %6.1f%%  %.3g ticks" % (names[k], 100 * d[k] / tot, d[k]))

"""Independent pin of the RANSAC oracle: the C1 (Lund Door, 66 pairs) verifier results of the round-2 oracle.

Round 4 rewrote oracle/ransac.c to mirror the kernel's operations (Householder-QR null space, explicit fma placement,
the LO refit's sums in the device's wave-reduction order, inverse iteration instead of Jacobi), then regenerated
lund_door/oracle_c1.npz from the rewritten oracle. The GPU is tested bit-exact against that file, i.e. against a
restatement of itself. This fixture keeps the verifier outputs of the oracle as it stood at commit dd09023 (MSAC model
selection, full-pivot Gauss-Jordan null space, cyclic Jacobi LO eigenvectors, compiler-chosen FMA placement) on the
same putatives, so tests/test_oracle_verifier.py can check that later oracle edits do not move the results:
equal inlier counts and masks, R and t within 2e-3 degrees.

    python tests/golden/make_prev_oracle_c1.py      (needs the git history; writes lund_door/oracle_c1_prev.npz)
"""
import io
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
COMMIT = "dd09023"

if __name__ == "__main__":
    blob = subprocess.run(["git", "-C", REPO, "show", f"{COMMIT}:tests/golden/lund_door/oracle_c1.npz"],
                          check=True, capture_output=True).stdout
    z = np.load(io.BytesIO(blob))
    np.savez_compressed(os.path.join(HERE, "lund_door", "oracle_c1_prev.npz"), commit=np.array(COMMIT),
                        pairs=z["pairs"], match_count=z["match_count"], status=z["status"], n_inliers=z["n_inliers"],
                        R=z["R"], t=z["t"], masks=np.packbits(z["masks"]))

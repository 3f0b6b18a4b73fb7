"""Front-end cache entries written BY THE REFERENCE'S OWN CACHERS (run in the build container only; the GPU box and the
CPU tests read the committed files, never the reference).

The reference's cacher modules are imported from /root/reference with the third-party modules this image lacks
(cv2, gtsam, dask, h5py, open3d, ...) stubbed as empty attribute-bags: none of the code that runs
here touches them -- the cachers compute their sha1 keys with hashlib (gtsfm/utils/cache.py:11-20) and write with
gtsfm/utils/io.py:626-630 (pickle.dump into a BZ2File); the payloads are gtsfm.common.keypoints.Keypoints,
numpy arrays and gtsfm.common.two_view_estimation_report.TwoViewEstimationReport, all pure Python / numpy. The
wrapped detector / matcher / estimator return fixed data (the reference's own Lund Door SIFT fixture,
tests/data/set1_lund_door/features, first 300 keypoints); the cachers do the rest exactly as the reference does:

- detector_descriptor/<SIFTDetectorDescriptor_key>.pbz2 -- DetectorDescriptorCacher.detect_and_describe
  (detector_descriptor_cacher.py:71-95) on a 48 x 64 crop of DSC_0001 named "DSC_0001.JPG";
- matcher/<key>.pbz2 -- MatcherCacher.match (matcher_cacher.py:127-192) on the two keypoint sets;
- two_view_estimator/<key>.pbz2 -- TwoViewEstimatorCacher.run_2view (two_view_estimator_cacher.py:83-114) with a
  failed verification (R, U None; the gtsam Rot3 / Unit3 of a successful entry cannot be made without gtsam).
The inputs needed to recompute the keys are saved beside them (inputs.npz). tests/test_cacher_reference_files.py
reads these files with this package's cachers (hits, no recomputation) and writes entries that the reference's
loader (here: pickle with the reference module names mapped to stand-ins) reads back.

    python tests/golden/make_reference_cache_fixtures.py
"""
import importlib.abc
import importlib.machinery
import os
import shutil
import sys
import types
from pathlib import Path

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
OUT = Path(HERE) / "reference_cache"
CANDIDATES = ("cv2", "gtsam", "dask", "distributed", "h5py", "open3d", "simplejson", "trimesh", "pycolmap", "hydra",
              "omegaconf", "kornia", "pydegensac", "matplotlib", "mayavi", "plotly", "graphviz", "networkx",
              "seaborn", "colour", "gdown", "kaggle", "rtree", "shapely", "boto3", "gtsfm_bindings")


def _missing(name):
    import importlib.util

    try:
        return importlib.util.find_spec(name) is None
    except (ImportError, ValueError):
        return True


STUBBED = {n for n in CANDIDATES if _missing(n)}


class _Bag(types.ModuleType):
    """A stand-in module: every attribute is another bag; classes derived from it are plain classes."""

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        if name[:1].isupper():  # a class-like name: a real (empty) class, usable as a base or annotation
            cls = type(name, (object,), {"__init__": lambda self, *a, **k: None})
            setattr(self, name, cls)
            return cls
        sub = _Bag(f"{self.__name__}.{name}")
        setattr(self, name, sub)
        return sub

    def __call__(self, *a, **k):
        return _Bag("call")

    def __mro_entries__(self, bases):
        return (object,)


class _StubFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    """Stubs the listed third-party modules that are not installed."""

    def find_spec(self, name, path, target=None):
        if any(name == s or name.startswith(s + ".") for s in STUBBED):
            return importlib.machinery.ModuleSpec(name, self, is_package=True)
        return None

    def create_module(self, spec):
        m = _Bag(spec.name)
        m.__path__ = []
        return m

    def exec_module(self, module):
        pass


def main():
    sys.meta_path.insert(0, _StubFinder())
    sys.path.insert(0, REF)
    import gtsfm.frontend.cacher.detector_descriptor_cacher as ddc
    import gtsfm.frontend.cacher.matcher_cacher as mc
    import gtsfm.two_view_estimator_cacher as tvc
    from gtsfm.common.image import Image
    from gtsfm.common.keypoints import Keypoints
    from gtsfm.common.two_view_estimation_report import TwoViewEstimationReport

    if OUT.exists():
        shutil.rmtree(OUT)
    for mod in (ddc, mc, tvc):
        mod.CACHE_ROOT_PATH = OUT

    fx = np.load(os.path.join(HERE, "lund_door_sift_fixture_0.npz"))
    print({k: fx[k].shape for k in fx.files})
    coords0 = fx["xy"][:300].astype(np.float64)
    scales0 = fx["scales"][:300].astype(np.float64)
    resp0 = fx["responses"][:300].astype(np.float64)
    desc = np.load(os.path.join(HERE, "lund_door_descriptors.npz"))
    d0 = desc["d0"][:300].astype(np.float32)
    d1 = desc["d1"][:300].astype(np.float32)
    rng = np.random.default_rng(5)
    coords1 = coords0 + rng.normal(0, 3, coords0.shape)
    kp0 = Keypoints(coordinates=coords0, scales=scales0, responses=resp0)
    kp1 = Keypoints(coordinates=coords1, scales=scales0.copy(), responses=resp0.copy())

    from PIL import Image as PILImage

    gray = np.asarray(PILImage.open(os.path.join(HERE, "lund_door_DSC_0001_gray.png")))
    crop = np.ascontiguousarray(np.repeat(gray[600:648, 400:464, None], 3, axis=2))
    image = Image(value_array=crop, exif_data=None, file_name="DSC_0001.JPG")

    class SIFTDetectorDescriptor:  # the wrapped plugin's class name is part of the reference's key
        max_keypoints = 5000

        def detect_and_describe(self, im):
            return kp0, d0

    det = ddc.DetectorDescriptorCacher(SIFTDetectorDescriptor())
    det.detect_and_describe(image)

    matches = np.array([[i, (i * 7) % 300] for i in range(0, 300, 3)], dtype=np.uint32)

    class TwoWayMatcher:
        def match(self, *a, **k):
            return matches

    m = mc.MatcherCacher(TwoWayMatcher())
    m.match(kp0, kp1, d0, d1, crop.shape, crop.shape)

    report = TwoViewEstimationReport(inlier_ratio_est_model=0.0, num_inliers_est_model=0,
                                     v_corr_idxs=np.array([], dtype=np.uint64))
    two_view_out = (None, None, np.array([], dtype=np.uint64), report, report, report)

    class _Estimator:
        def run_2view(self, *a, **k):
            return two_view_out

    t = tvc.TwoViewEstimatorCacher(_Estimator())
    t.run_2view(kp0, kp1, matches, None, None, None, None, None)

    np.savez_compressed(OUT / "inputs.npz", coords0=coords0, scales0=scales0, resp0=resp0, coords1=coords1, d0=d0,
                        d1=d1, crop=crop, matches=matches)
    for p in sorted(OUT.rglob("*.pbz2")):
        print(p.relative_to(OUT), p.stat().st_size)
    print("stubbed:", sorted(STUBBED))


if __name__ == "__main__":
    main()

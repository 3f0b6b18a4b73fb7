"""gtsfm_amd — MI355X-native (gfx950) GTSfM two-view front-end.

Drop-in replacements for the reference's front-end plugins (detector-descriptor, matcher, verifier,
correspondence generator, two-view estimator), backed by hand-written HIP kernels in libgtsfm_hip.so.
"""
__version__ = "0.1.0"

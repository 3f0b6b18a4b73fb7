"""Cache keys of the front-end cachers (reference gtsfm/utils/cache.py:11-20).

The keys are the reference's: sha1 over `"{file_name}_{width}_{height}"` followed by sha1 of the image bytes for
detector-descriptor entries, sha1 of a concatenated numpy array for matcher and two-view entries. A cache directory
written by the reference's cachers therefore resolves to the same file names here, and vice versa.
"""
import hashlib

import numpy as np

from gtsfm_amd.common.image import Image


def generate_hash_for_image(image: Image) -> str:
    """Hash of the image name, shape and content (cache.py:11-15)."""
    return hashlib.sha1(
        "{}_{}_{}".format(image.file_name, image.width, image.height).encode()
    ).hexdigest() + generate_hash_for_numpy_array(image.value_array)


def generate_hash_for_numpy_array(input: np.ndarray) -> str:
    """sha1 of the array's buffer (cache.py:18-20); the array must be C-contiguous, as `hashlib` requires."""
    return hashlib.sha1(input).hexdigest()

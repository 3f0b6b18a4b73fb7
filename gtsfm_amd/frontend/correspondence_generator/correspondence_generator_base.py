"""Correspondence-generator interface (reference: frontend/correspondence_generator/correspondence_generator_base.py).

`client` is accepted for signature compatibility with the reference's Dask call site (gtsfm_runner_base.py:326-331)
and is not used: the MI355X path batches all images and pairs on the device instead of fanning out tasks.
"""
import abc
from typing import Dict, List, Tuple

import numpy as np

from gtsfm_amd.common.keypoints import Keypoints


class CorrespondenceGeneratorBase(metaclass=abc.ABCMeta):
    @abc.abstractmethod
    def generate_correspondences(
        self, client, images: List, image_pairs: List[Tuple[int, int]]
    ) -> Tuple[List[Keypoints], Dict[Tuple[int, int], np.ndarray]]:
        """Returns keypoints of every image and putative (M, 2) uint32 correspondences of every requested pair."""

"""Image-pair generation for the front-end (mirrors gtsfm/retriever/image_pairs_generator.py:17-47).

The reference scatters the global descriptor to Dask workers, submits one describe() per image, gathers the (D,)
arrays to the client and hands them to the retriever. Here the descriptors of a NetVLADGlobalDescriptor (optionally
behind the reference's GlobalDescriptorCacher: hits from disk, misses batched and written back) are computed in
batched launches and stay in HBM; the NetVLAD retriever's similarity GEMM and top-k selection read them there
(gtsfm_amd/retriever/netvlad_retriever.py), so only the pair list comes back to the host.
"""
from __future__ import annotations

from pathlib import Path
from typing import List, Optional, Tuple

import numpy as np
import torch

from gtsfm_amd.common.image import Image
from gtsfm_amd.frontend.cacher.global_descriptor_cacher import GlobalDescriptorCacher
from gtsfm_amd.frontend.global_descriptor.global_descriptor_base import GlobalDescriptorBase
from gtsfm_amd.frontend.global_descriptor.netvlad_global_descriptor import NetVLADGlobalDescriptor
from gtsfm_amd.retriever.retriever_base import RetrieverBase


def _resolve(obj):
    return obj.result() if hasattr(obj, "result") and callable(obj.result) else obj


class ImagePairsGenerator:
    def __init__(self, retriever: RetrieverBase, global_descriptor: Optional[GlobalDescriptorBase] = None):
        self._global_descriptor: Optional[GlobalDescriptorBase] = global_descriptor
        self._retriever: RetrieverBase = retriever

    def __repr__(self) -> str:
        return f"""
            ImagePairGenerator:
                {self._global_descriptor}
                {self._retriever}
        """

    def global_descriptors(self, images: List[Image]):
        """(n, D) device tensor for the HIP NetVLAD (cacher-wrapped or not), else a list of (D,) arrays."""
        gd = self._global_descriptor
        cacher = gd if type(gd) is GlobalDescriptorCacher else None
        inner = cacher.wrapped if cacher is not None else gd
        if type(inner) is not NetVLADGlobalDescriptor:
            return [gd.describe(im) for im in images]
        if cacher is None:
            return inner.describe_device(images)
        hits = [cacher.cache_lookup(im) for im in images]
        miss = [i for i, h in enumerate(hits) if h is None]
        fresh = inner.describe_device([images[i] for i in miss]) if miss else None
        dim = fresh.shape[1] if fresh is not None else int(np.asarray(hits[0]).size)
        out = torch.empty((len(images), dim), dtype=torch.float32, device=torch.device("cuda"))
        if miss:
            host = fresh.cpu().numpy()
            for j, i in enumerate(miss):
                cacher.cache_store(images[i], host[j].copy())
            out[torch.tensor(miss, dtype=torch.long, device=out.device)] = fresh
        hit_idx = [i for i, h in enumerate(hits) if h is not None]
        if hit_idx:
            arr = np.stack([np.asarray(hits[i], np.float32).reshape(-1) for i in hit_idx])
            out[torch.tensor(hit_idx, dtype=torch.long, device=out.device)] = torch.from_numpy(arr).to(out.device)
        return out

    def generate_image_pairs(self, client, images: List, image_fnames: List[str],
                             plots_output_dir: Optional[Path] = None) -> List[Tuple[int, int]]:
        """image_pairs_generator.py:29-47 (client unused: the batching replaces the Dask fan-out)."""
        descriptors = None
        if self._global_descriptor is not None:
            descriptors = self.global_descriptors([_resolve(im) for im in images])
        return self._retriever.get_image_pairs(global_descriptors=descriptors, image_fnames=image_fnames,
                                               plots_output_dir=plots_output_dir)

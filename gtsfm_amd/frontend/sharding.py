"""Multi-GPU layout of the all-pairs front-end: one process per GPU, one exchange step.

The reference fans the front-end out as Dask tasks, one per image and one per pair
(det_desc_correspondence_generator.py:64-80, two_view_estimator.py:568-584), and pickles ~2 MiB of features into
every pair task. Here each rank owns a fixed share instead:

- extraction: image i -> rank i mod world (rank-local order i // world);
- exchange: ONE all-gather of the fixed-size per-rank feature block (descriptors, keypoint xy, counts packed into one
  byte buffer), padded to `n_per = ceil(n / world)` images per rank, so the gathered tensors are rank-major: image i
  sits in global slot `(i mod world) * n_per + i // world`;
- matching + verification: the (i1, i2) pair list cut into runs of consecutive pairs that share i1 and the block
  i2 // PAIR_BLOCK (the distance GEMM's pair groups, device.pair_groups: up to 4 pairs that share the register
  operand), the runs dealt round-robin (run r to rank r mod world). Contiguous blocks of the list left the ranks
  unequal: its tail holds the close (many-match) pairs of the last images, so at C4 on 8 ranks rank 7's RANSAC took
  74 ms against rank 0's 44 (`profiles/r05aj_*`). Dealing single pairs round-robin (round 5) balanced them but split
  every pair group across ranks (at 2 / 4 ranks a rank's groups were half / a quarter full, so the matcher re-read
  its register operand per pair); whole runs keep the groups and the balance. Every pair keeps its global index,
  which keys the RANSAC sampler: a pair's result does not depend on the world size.

Nothing here is GPU specific: the same functions run on CPU tensors under the gloo backend (tests/test_sharding.py).
"""
from __future__ import annotations

import math
from typing import Optional, Sequence, Tuple

import numpy as np
import torch


def images_per_rank(n_img: int, world: int) -> int:
    return int(math.ceil(n_img / max(world, 1)))


def local_images(n_img: int, world: int, rank: int) -> np.ndarray:
    """Original indices of the images rank `rank` extracts, in its local order."""
    return np.arange(rank, n_img, world, dtype=np.int64)


def global_slots(n_img: int, world: int) -> np.ndarray:
    """slot[i] = row of image i in the gathered (world * n_per, ...) feature tensors."""
    i = np.arange(n_img, dtype=np.int64)
    return (i % world) * images_per_rank(n_img, world) + i // world


def all_pairs(n_img: int) -> np.ndarray:
    """Every (i1 < i2) pair in lexicographic order, (P, 2) int64 (the exhaustive pair list of the reference)."""
    i1, i2 = np.triu_indices(n_img, k=1)
    return np.stack([i1, i2], axis=1).astype(np.int64)


PAIR_BLOCK = 4  # i2 block of the distance GEMM's pair groups (device.pair_groups at the default max group of 4)


def pair_runs(pairs: np.ndarray, block: int = PAIR_BLOCK) -> np.ndarray:
    """Run id of every pair: consecutive pairs with the same (i1, i2 // block) share a run."""
    pairs = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
    if len(pairs) == 0:
        return np.zeros(0, dtype=np.int64)
    key = pairs[:, 0] * (int(pairs[:, 1].max()) // block + 1) + pairs[:, 1] // block
    return np.r_[0, np.cumsum(key[1:] != key[:-1])].astype(np.int64)


def rank_pairs(pairs: np.ndarray, world: int, rank: int, block: int = PAIR_BLOCK) -> np.ndarray:
    """Positions (into `pairs`) of the pairs rank `rank` matches and verifies, in list order: the runs of pair_runs
    dealt in list order, each to the rank holding the fewest pairs so far (lowest rank on ties) -- round-robin while
    the runs are equal, and never more than one run (<= block pairs) apart when they are not."""
    world = max(world, 1)
    if world == 1:
        return np.arange(len(pairs), dtype=np.int64)
    return np.flatnonzero(run_owners(pairs, world, block) == rank).astype(np.int64)


def run_owners(pairs: np.ndarray, world: int, block: int = PAIR_BLOCK) -> np.ndarray:
    """Owning rank of every pair under rank_pairs' dealing."""
    run = pair_runs(pairs, block)
    if len(run) == 0:
        return run
    sizes = np.bincount(run)
    owner_of_run = np.empty(len(sizes), dtype=np.int64)
    load = [0] * world
    for r, sz in enumerate(sizes.tolist()):
        k = min(range(world), key=load.__getitem__)
        owner_of_run[r] = k
        load[k] += sz
    return owner_of_run[run]


def pack_features(tensors: Sequence[torch.Tensor], n_per: int,
                  wire: Optional[Sequence[Optional[torch.dtype]]] = None) -> Tuple[torch.Tensor, list]:
    """One rank's feature tensors padded to n_per rows and packed byte-wise into a single block (each field 16-byte
    aligned, in its wire dtype). Returns (block (off,) uint8, layout) for unpack_features."""
    fields, layout, off = [], [], 0
    for i, t in enumerate(tensors):
        dtype = t.dtype
        if wire is not None and wire[i] is not None:
            t = t.to(wire[i])
        pad = n_per - t.shape[0]
        if pad < 0:
            raise ValueError(f"rank holds {t.shape[0]} images, more than n_per={n_per}")
        if pad:
            t = torch.cat([t, t.new_zeros((pad,) + tuple(t.shape[1:]))])
        raw = t.contiguous().view(-1).view(torch.uint8)
        nbytes = raw.numel()
        layout.append((off, nbytes, t.dtype, tuple(t.shape), dtype))
        fields.append(raw)
        off += -(-nbytes // 16) * 16
    block = torch.zeros(off, dtype=torch.uint8, device=tensors[0].device)
    for raw, (o, nb, _, _, _) in zip(fields, layout):
        block[o: o + nb] = raw
    return block, layout


def unpack_features(g: torch.Tensor, layout: list) -> Tuple[torch.Tensor, ...]:
    """(world, off) gathered blocks -> the rank-major (world * n_per, ...) feature tensors, cast back."""
    world = g.shape[0]
    out = []
    for o, nb, wdt, shape, dtype in layout:
        f = g[:, o: o + nb].contiguous().view(wdt).view((world * shape[0],) + shape[1:])
        out.append(f if f.dtype == dtype else f.to(dtype))
    return tuple(out)


def allgather_features(tensors: Sequence[torch.Tensor], n_per: int,
                       group: Optional[torch.distributed.ProcessGroup] = None,
                       wire: Optional[Sequence[Optional[torch.dtype]]] = None,
                       exchange=None) -> Tuple[torch.Tensor, ...]:
    """Pads each rank's (n_local, ...) feature tensors to n_per rows and all-gathers them rank-major, in ONE
    collective: the tensors are packed byte-wise into a single per-rank block (each field 16-byte aligned), gathered
    with one all_gather_into_tensor, and unpacked as views of the gathered buffer.

    wire[i] (optional) is the dtype tensor i travels in; it is cast back afterwards, so the caller must only name a
    lossless one: SIFT descriptors are integers in [0, 255], so u8 carries them exactly (2048 x 128 B per image
    instead of 4x that in f32). With world == 1 the inputs are returned unchanged.

    exchange (optional): an EmulatedAllGather standing in for the collective (one process running one rank's share
    of a larger job on one GPU); the packing and unpacking around it are the real ones.
    """
    if exchange is None:
        world = torch.distributed.get_world_size(group) if torch.distributed.is_initialized() else 1
        if world == 1:
            return tuple(tensors)
        exchange = CollectiveAllGather(group)
    block, layout = pack_features(tensors, n_per, wire)
    return unpack_features(exchange(block), layout)


class CollectiveAllGather:
    """The exchange's collective: one all_gather_into_tensor of the packed per-rank blocks over the process group
    (RCCL over xGMI under the "nccl" backend). allgather_features uses it for world > 1; passed explicitly as
    `exchange`, it runs the collective at any world size, including 1 (tests/test_rccl_gpu.py drives the RCCL path
    on a one-GPU box that way)."""

    def __init__(self, group: Optional[torch.distributed.ProcessGroup] = None):
        self.group = group

    def __call__(self, block: torch.Tensor) -> torch.Tensor:
        world = torch.distributed.get_world_size(self.group)
        off = block.numel()
        g = torch.empty(world * off, dtype=torch.uint8, device=block.device)
        torch.distributed.all_gather_into_tensor(g, block, group=self.group)
        return g.view(world, off)


class EmulatedAllGather:
    """The all-gather of rank `rank` in a `world`-rank job, emulated in one process on one GPU: the other ranks'
    packed blocks were produced beforehand (their extraction, untimed) and sit in `others` (world, off); a call copies
    them and this rank's fresh block into the gathered buffer, i.e. the bytes the collective would write here. The
    xGMI transfer itself is not included (bench.py --emulate-world reports that)."""

    def __init__(self, others: torch.Tensor, rank: int):
        self.others, self.rank = others, rank

    def __call__(self, block: torch.Tensor) -> torch.Tensor:
        if block.numel() != self.others.shape[1]:
            raise ValueError(f"block of {block.numel()} bytes, the emulated job packs {self.others.shape[1]}")
        g = torch.empty_like(self.others)
        g.copy_(self.others)
        g[self.rank].copy_(block)
        return g


def gather_pair_results(local: torch.Tensor, pairs: np.ndarray,
                        group: Optional[torch.distributed.ProcessGroup] = None) -> torch.Tensor:
    """Reassembles a per-pair result tensor (rank r holds the pairs rank_pairs(pairs, .., r), in that order) into
    pair order everywhere.

    Used only where a caller wants every rank to hold every pair's compact result (R, t, counts); the bench and the
    batched drop-ins copy each rank's results to the host instead.
    """
    world = torch.distributed.get_world_size(group) if torch.distributed.is_initialized() else 1
    if world == 1:
        return local
    owned = [rank_pairs(pairs, world, r) for r in range(world)]
    per = max(len(o) for o in owned)
    pad = per - local.shape[0]
    buf = torch.cat([local, local.new_zeros((pad,) + tuple(local.shape[1:]))]) if pad else local.contiguous()
    g = torch.empty((world * per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    torch.distributed.all_gather_into_tensor(g, buf, group=group)
    g = g.view((world, per) + tuple(local.shape[1:]))
    out = local.new_empty((len(pairs),) + tuple(local.shape[1:]))
    for r, o in enumerate(owned):
        out[torch.from_numpy(o).to(out.device)] = g[r, : len(o)]
    return out

"""One process per GPU: the launcher behind `bench.py --gpus N` and the rank-side setup every rank runs.

The reference spreads the front-end over Dask worker processes on a LocalCluster
(gtsfm/runner/gtsfm_runner_base.py:287-296: `LocalCluster(n_workers, threads_per_worker=1)` + `Client`). Here each
rank is one OS process owning one GPU, started BEFORE anything touches the GPU:

- `spawn_ranks(n, script, argv)` starts n fresh child interpreters on `script` with RANK / LOCAL_RANK /
  WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set (torchrun's environment contract), waits for all of them
  and returns the first non-zero exit status. When one rank fails, the others are terminated (they would otherwise
  block in a collective). The parent never initialises HIP, so no process that touched the GPU is ever replaced.
- `init_rank(backend)` reads that environment (or defaults to a single rank), binds the rank to its GPU and joins
  the process group: `nccl` (= RCCL over xGMI on ROCm) on the GPU, `gloo` on CPU for tests.

`python -m torch.distributed.run --nproc-per-node N bench.py --gpus N` sets the same variables, so bench.py runs
unchanged under either launcher.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(rank: int, world: int, port: int, base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # the host driver supports dmabuf IPC only
    return env


def spawn_ranks(n_ranks: int, script: str, argv: Sequence[str], env: Optional[Dict[str, str]] = None,
                poll_s: float = 0.2) -> int:
    """Runs `python script *argv` as n_ranks ranks of one job; returns 0 or the first failing rank's status."""
    if n_ranks < 1:
        raise ValueError("n_ranks must be >= 1")
    port = free_port()
    procs: List[subprocess.Popen] = []
    for r in range(n_ranks):
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=rank_env(r, n_ranks, port, env)))
    rc = 0
    try:
        while True:
            states = [p.poll() for p in procs]
            failed = [s for s in states if s not in (None, 0)]
            if failed:
                rc = failed[0]
                break
            if all(s == 0 for s in states):
                break
            time.sleep(poll_s)
    finally:
        for p in procs:  # only the processes started here
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc


@dataclass
class RankInfo:
    rank: int
    world: int
    local_rank: int
    device: "object"  # torch.device


def launched_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def init_rank(backend: str = "nccl") -> RankInfo:
    """Binds this process to its GPU (LOCAL_RANK) and joins the job's process group when WORLD_SIZE > 1.

    backend "nccl" = RCCL on the MI355X; "gloo" = CPU tensors (tests, rehearsals without a GPU).
    """
    import torch
    import torch.distributed as dist

    world = launched_world()
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "gloo":
        dev = torch.device("cpu")
    else:
        n_dev = torch.cuda.device_count()
        if local_rank >= n_dev:
            raise RuntimeError(f"rank {rank}: LOCAL_RANK {local_rank} but only {n_dev} GPU(s) visible")
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
    if world > 1 and not dist.is_initialized():
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group(backend, device_id=dev)
    if world > 1 and dist.get_world_size() != world:
        raise RuntimeError(f"WORLD_SIZE={world} but the process group has {dist.get_world_size()} ranks")
    return RankInfo(rank, world, local_rank, dev)


def finish_rank(info: RankInfo) -> None:
    import torch.distributed as dist

    if info.world > 1 and dist.is_initialized():
        dist.destroy_process_group()

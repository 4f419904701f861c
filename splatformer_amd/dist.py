"""Multi-GPU orchestration of the hot path: one process per GPU, scenes sharded across ranks.

Within a scene the path does not shard (pooling needs a global unique/sort per stage), so the unit of
parallelism is the scene:
- evaluation: contiguous chunks of the scene list per rank, the last rank taking the remainder
  (reference dataset/GS.py:54-67), no exchange on the data path; the metrics are summed to rank 0 with
  `reduce` and divided by the global image count (train.py:170-176);
- timing: barrier + max over ranks (the bench contract).

Training (config D): one scene per rank per micro-step; the only exchanges are the gradient bucket
all-reduce per optimiser step (DDP average, one flat fp32 bucket) and SyncBatchNorm's per-layer column
sums (train.py:404) -- both below.

Backend "nccl" is RCCL on ROCm; the CPU tests drive the same code with "gloo".
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as tdist


def env_rank() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str = "nccl") -> bool:
    """Initialise the process group when WORLD_SIZE > 1 (rendezvous on 127.0.0.1 unless set)."""
    rank, world, _ = env_rank()
    if world <= 1 or tdist.is_initialized():
        return tdist.is_initialized()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    tdist.init_process_group(backend, rank=rank, world_size=world)
    return True


def world() -> Tuple[int, int]:
    if tdist.is_available() and tdist.is_initialized():
        return tdist.get_rank(), tdist.get_world_size()
    return 0, 1


def scene_chunk(num_scenes: int, rank: int, world_size: int) -> List[int]:
    """dataset/GS.py:57-67: chunk = n // world; rank r gets [r*chunk, (r+1)*chunk), the last rank the rest."""
    scenes = list(range(num_scenes))
    chunk = num_scenes // world_size
    if rank == world_size - 1:
        return scenes[rank * chunk:]
    return scenes[rank * chunk:(rank + 1) * chunk]


def barrier() -> None:
    if tdist.is_available() and tdist.is_initialized():
        tdist.barrier()


def max_over_ranks(value: float, device: Optional[torch.device] = None) -> float:
    """Max of a host scalar over all ranks (the bench's wall-clock rule)."""
    if not (tdist.is_available() and tdist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item())


def reduce_metrics(metric_sums: Dict[str, torch.Tensor], num_images: int, num_scenes: int,
                   device: Optional[torch.device] = None) -> Dict[str, float]:
    """train.py:170-176: sum every metric, the image and the scene counts to rank 0; rank 0 returns the
    per-image means (other ranks return {})."""
    rank, ws = world()
    dev = device if device is not None else torch.device("cpu")
    n_img = torch.tensor([num_images], dtype=torch.float64, device=dev)
    n_scn = torch.tensor([num_scenes], dtype=torch.float64, device=dev)
    sums = {k: v.detach().to(dev, torch.float64).reshape(1).clone() for k, v in metric_sums.items()}
    if ws > 1:
        tdist.reduce(n_img, dst=0)
        tdist.reduce(n_scn, dst=0)
        for k in sorted(sums):
            tdist.reduce(sums[k], dst=0)
    if rank != 0:
        return {}
    out = {k: float(v.item() / n_img.item()) for k, v in sums.items()}
    out["num_images"] = int(n_img.item())
    out["num_scenes"] = int(n_scn.item())
    return out


def allreduce_mean_(flat: torch.Tensor, group=None) -> torch.Tensor:
    """DDP gradient averaging on one flat bucket: sum over ranks, divide by the world size (in place)."""
    if not (tdist.is_available() and tdist.is_initialized()):
        return flat
    ws = tdist.get_world_size(group)
    if ws > 1:
        tdist.all_reduce(flat, group=group)
        flat.div_(ws)
    return flat


def allreduce_sum_(t: torch.Tensor, group=None) -> torch.Tensor:
    """SyncBatchNorm statistics: per-column sums (and the row count) summed over ranks, in place."""
    if group is not None or (tdist.is_available() and tdist.is_initialized()):
        if tdist.get_world_size(group) > 1:
            tdist.all_reduce(t, group=group)
    return t

"""Frame-batch sharding across GPUs (one process per GPU, torch.distributed; "nccl" = RCCL).

Frames are independent units, so the steady-state path has no data-path
collective: rank r owns frames [r*F, (r+1)*F) already resident in its HBM, and only the
timing (max over ranks) and the small per-frame result headers cross ranks. For the C4
composition the north star describes (a root holding the whole batch), `scatter_frames`
moves each rank's share with one scatter and `gather_headers` brings the per-frame results
back with one gather; over xGMI that is one point-to-point transfer per peer.
"""
import os

import torch
import torch.distributed as dist


def world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def frame_range(rank: int, frames_per_rank: int) -> range:
    """Global frame indices owned by `rank` (weak scaling: fixed frames per rank)."""
    return range(rank * frames_per_rank, (rank + 1) * frames_per_rank)


def max_over_ranks(value: float, device) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def scatter_frames(all_frames, frames_per_rank: int, frame_bytes: int, device, src: int = 0):
    """Root holds (world * F, frame_bytes) uint8 frames; every rank receives its (F, frame_bytes)."""
    ws = dist.get_world_size()
    out = torch.empty((frames_per_rank, frame_bytes), dtype=torch.uint8, device=device)
    chunks = list(all_frames.chunk(ws, dim=0)) if dist.get_rank() == src else None
    dist.scatter(out, chunks, src=src)
    return out


def gather_headers(headers, dst: int = 0):
    """Gather each rank's (F, 8) int32 per-frame result headers to `dst` as (world * F, 8)."""
    ws = dist.get_world_size()
    bufs = [torch.empty_like(headers) for _ in range(ws)] if dist.get_rank() == dst else None
    dist.gather(headers, bufs, dst=dst)
    return torch.cat(bufs, 0) if bufs is not None else None

"""Frame sharding across GPUs (one process per GPU) and the gather of the
encoded per-frame streams to rank 0.

Frames are the reference's only unit of parallelism (encoder.lpr:1449,
DoParallelLocalProc over frame indices) and share nothing
(encoder.lpr:1433-1447), so the stream shards into contiguous frame ranges,
one per rank, with no exchange on the data path.  The only collective is the
final gather of each rank's concatenated TFrame.SaveStream bytes
(encoder.lpr:1181-1215 writes frames in order): an all-gather of the byte
counts, then one padded all-gather of uint8 tensors (RCCL over xGMI on the
GPU box; gloo in the CPU tests).
"""
from __future__ import annotations

from typing import Sequence


def frame_range(frame_count: int, rank: int, world_size: int) -> tuple[int, int]:
    """Contiguous [begin, end) frame range of `rank` (frames ~equal length)."""
    if world_size <= 0 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} / world size {world_size}")
    return (frame_count * rank) // world_size, (frame_count * (rank + 1)) // world_size


def frame_range_weighted(weights: Sequence[int], rank: int, world_size: int) -> tuple[int, int]:
    """Contiguous range balancing sum(weights) (chunk counts) across ranks."""
    total = sum(weights)
    bounds = [0]
    acc = 0
    r = 1
    for i, w in enumerate(weights):
        acc += w
        while r < world_size and acc * world_size >= total * r:
            bounds.append(i + 1)
            r += 1
    while len(bounds) < world_size:
        bounds.append(len(weights))
    bounds.append(len(weights))
    return bounds[rank], bounds[rank + 1]


def gather_streams(blob: bytes, group=None, device=None) -> bytes | None:
    """Concatenate every rank's bytes in rank order on rank 0 (None elsewhere).

    Sizes are all-gathered first, then one padded all-gather of uint8 tensors
    moves the payload (a single collective, sized for the largest shard)."""
    import torch
    import torch.distributed as dist

    ws = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = device if device is not None else torch.device("cpu")
    n = torch.tensor([len(blob)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(ws)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    cap = max(1, max(sizes))
    buf = torch.zeros(cap, dtype=torch.uint8, device=dev)
    if blob:
        buf[: len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    parts = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(ws)]
    dist.all_gather(parts, buf, group=group)
    if rank != 0:
        return None
    return b"".join(bytes(p[:s].cpu().numpy().tobytes()) for p, s in zip(parts, sizes))

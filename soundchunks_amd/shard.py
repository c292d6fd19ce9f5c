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


def bounds_range(starts, ends, chunk_size: int, channels: int, rank: int, world_size: int) -> tuple[int, int]:
    """This rank's LPT frame range from PrepareFrames' boundaries: frames are
    weighted by their chunkRefs count ((samples - 1) div ChunkSize + 1) x
    channels (encoder.lpr:467-485)."""
    import numpy as np

    st = np.asarray(starts, dtype=np.int64)
    en = np.asarray(ends, dtype=np.int64)
    chunks = ((en - st) // chunk_size + 1) * channels
    return frame_range_weighted(chunks.tolist(), rank, world_size)


def broadcast_bounds(starts, ends, group=None, device=None, src: int = 0):
    """Rank `src` ran PrepareFrames (the sequential frame-cut scan of the whole
    file, encoder.lpr:1399-1425); every rank gets its frame boundaries (one
    broadcast of the count, one of the int32 starts|ends)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    dev = device if device is not None else torch.device("cpu")
    n = torch.tensor([0 if starts is None else len(starts)], dtype=torch.int64, device=dev)
    dist.broadcast(n, src, group=group)
    buf = torch.empty(2 * int(n.item()), dtype=torch.int32, device=dev)
    if rank == src:
        buf.copy_(torch.from_numpy(np.concatenate([np.asarray(starts), np.asarray(ends)]).astype(np.int32)))
    dist.broadcast(buf, src, group=group)
    b = buf.cpu().numpy()
    return b[: len(b) // 2], b[len(b) // 2:]


def free_port() -> int:
    """A free TCP port on 127.0.0.1 for a rendezvous."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_workers(n: int, cmd: Sequence[str], env_extra: dict | None = None) -> int:
    """Launch `cmd` as n worker processes (RANK / LOCAL_RANK / WORLD_SIZE,
    rendezvous at 127.0.0.1 on a free port) and wait; the first non-zero exit
    ends the others.  Used by bench.py --gpus N before any GPU call."""
    import os
    import subprocess
    import time

    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **(env_extra or {}))
        procs.append(subprocess.Popen(list(cmd), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:  # a failed rank would leave the others waiting in a collective
                    q.terminate()
        time.sleep(0.05)
    return rc


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


def gather_files(blob: bytes, sizes: Sequence[int], group=None, device=None) -> list[bytes] | None:
    """Per-file streams of a sharded batch (gsc_encode_prepared_files): every
    rank holds `blob` = its frames' bytes, `sizes[f]` of them file f's.  Rank 0
    gets each file's bytes from all ranks in rank (= frame) order; one
    all-gather of the size tables, one padded all-gather of the blobs."""
    import numpy as np
    import torch
    import torch.distributed as dist

    ws = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = device if device is not None else torch.device("cpu")
    nf = len(sizes)
    t = torch.tensor(list(sizes), dtype=torch.int64, device=dev)
    tabs = [torch.zeros(nf, dtype=torch.int64, device=dev) for _ in range(ws)]
    dist.all_gather(tabs, t, group=group)
    whole = gather_streams(blob, group=group, device=device)
    if rank != 0:
        return None
    tabs = [np.asarray(x.cpu().numpy(), dtype=np.int64) for x in tabs]
    pieces = [[] for _ in range(nf)]
    o = 0
    for r in range(ws):
        for f in range(nf):
            n = int(tabs[r][f])
            pieces[f].append(whole[o:o + n])
            o += n
    return [b"".join(p) for p in pieces]

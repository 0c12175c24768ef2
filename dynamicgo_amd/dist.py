"""Multi-GPU plumbing for the batch transcoder.

Messages are independent, so a batch shards into contiguous ranges, one per
rank, with no data-path collective. The only exchange is the flattened
descriptor, broadcast once from rank 0 (RCCL over xGMI when the process group
is "nccl", gloo on CPU in tests) and created on each device from the received
bytes. One process per GPU; ranks read RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist


def shard_ranges(in_off: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """Contiguous message ranges balanced by cumulative JSON bytes: rank r gets
    messages [lo, hi) whose byte span starts nearest to r/world of the total."""
    off = np.asarray(in_off, dtype=np.uint64)
    n = len(off) - 1
    total = int(off[-1] - off[0])
    cuts = [0]
    for r in range(1, world):
        target = int(off[0]) + total * r // world
        k = int(np.searchsorted(off[:n], target, side="left"))
        cuts.append(max(cuts[-1], min(k, n)))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def broadcast_blob(blob: Optional[bytes], device: torch.device, src: int = 0) -> torch.Tensor:
    """Broadcast the descriptor blob from `src` to every rank; returns it as a
    uint8 tensor on `device` (device memory on GPUs: dg_desc_create_device
    consumes it without a host round trip)."""
    rank = dist.get_rank()
    nb = torch.tensor([len(blob) if rank == src else 0], dtype=torch.int64, device=device)
    dist.broadcast(nb, src)
    t = torch.empty(int(nb.item()), dtype=torch.uint8, device=device)
    if rank == src:
        t.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
    dist.broadcast(t, src)
    return t

"""One process per GPU for the many-sequence configuration.

Each rank owns one independent sequence (seed + rank): no collective in the data path.  The
only exchange is after the timed region: every rank's per-frame summary is gathered (RCCL
all_gather on GPU, gloo on CPU tests) and the step time is max-reduced.
"""
from __future__ import annotations

import os


def rank_env() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def sequence_seed(base: int, rank: int) -> int:
    """Seed of rank r's sequence (seed + rank)."""
    return (base + rank) & 0xFFFFFFFFFFFFFFFF


_cpu_collectives = False  # gloo: collectives on host copies (device tensors move through the CPU)


def init(backend: str, local_rank: int):
    """Initialise torch.distributed when WORLD_SIZE > 1; returns the module or None.  With gloo
    (CPU tests, and bench.py --rehearse-one-gpu: several ranks sharing one GPU, which RCCL refuses)
    the helpers below run the collectives on host copies."""
    global _cpu_collectives
    _, world, _ = rank_env()
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend)
        _cpu_collectives = True
    return dist


def max_over_ranks(value: float, device, dist) -> float:
    import torch

    t = torch.tensor([value], dtype=torch.float64, device="cpu" if _cpu_collectives else device)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_rows(rows, dist):
    """All-gather a same-shape tensor from every rank; returns a list ordered by rank."""
    import torch

    if dist is None:
        return [rows]
    src = rows.cpu() if _cpu_collectives else rows
    out = [torch.zeros_like(src) for _ in range(dist.get_world_size())]
    dist.all_gather(out, src)
    return [o.to(rows.device) for o in out] if _cpu_collectives else out


def barrier(dist) -> None:
    if dist is not None:
        dist.barrier()
